#!/usr/bin/env bash
run_observability_playbook() {
    local pb=playbooks/deploy-observability.yml
    [ "$kubernetes_platform" = "openshift" ] && pb=playbooks/deploy-observability-openshift.yml
    ansible-playbook -i "${INVENTORY_PATH}" "$pb" \
        --extra-vars "secret_name=${cluster_url} gpu_platform=${gpu_platform}" \
        --vault-password-file "$vault_pass_file"
}

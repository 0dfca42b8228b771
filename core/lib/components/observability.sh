#!/usr/bin/env bash
run_observability_playbook() {
    local pb=playbooks/deploy-observability.yml
    [ "$kubernetes_platform" = "openshift" ] && pb=playbooks/deploy-observability-openshift.yml
    ansible-playbook -i "${INVENTORY_PATH}" "$pb" \
        --extra-vars "secret_name=${cluster_url} cert_file=${cert_file} key_file=${key_file} gpu_platform=${gpu_platform} kubernetes_platform=${kubernetes_platform} observability_stack_chart_version=${observability_stack_chart_version}" \
        --vault-password-file "$vault_pass_file"
}

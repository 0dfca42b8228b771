#!/usr/bin/env bash
run_genai_gateway_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-genai-gateway.yml \
        --extra-vars "secret_name=${cluster_url} cert_file=${cert_file} key_file=${key_file} kubernetes_platform=${kubernetes_platform} genai_gateway_trace_chart_version=${genai_gateway_trace_chart_version}" \
        --vault-password-file "$vault_pass_file"
}

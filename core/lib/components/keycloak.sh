#!/usr/bin/env bash
run_keycloak_playbook() {
    local kc_vars="secret_name=${cluster_url} cert_file=${cert_file} key_file=${key_file} keycloak_admin_user=${keycloak_admin_user} keycloak_admin_password=${keycloak_admin_password} keycloak_client_id=${keycloak_client_id} kubernetes_platform=${kubernetes_platform}"
    local pin_vars="keycloak_chart_version=${keycloak_chart_version} apisix_chart_version=${apisix_chart_version}"
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-keycloak-controller.yml --extra-vars "${kc_vars}" --vault-password-file "$vault_pass_file" || return 1
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-keycloak-tls-cert.yml --extra-vars "${kc_vars} ${pin_vars}" --vault-password-file "$vault_pass_file"
}

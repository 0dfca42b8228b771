#!/usr/bin/env bash
run_ingress_controller_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-ingress-controller.yml \
        --extra-vars "secret_name=${cluster_url} cert_file=${cert_file} key_file=${key_file} kubernetes_platform=${kubernetes_platform} ingress_controller=${ingress_controller}"
}

#!/usr/bin/env bash
run_deploy_amd_gpu_operator_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-amd-gpu-operator.yml --extra-vars amd_gpu_operator=${amd_gpu_operator}
}

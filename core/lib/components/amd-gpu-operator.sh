#!/usr/bin/env bash
# Pins from inventory/metadata/inference-metadata.cfg: the operator chart version and the
# amdgpu driver version the DeviceConfig installs when the in-cluster driver is enabled.
run_deploy_amd_gpu_operator_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-amd-gpu-operator.yml \
        --extra-vars "amd_gpu_operator_version=${amd_gpu_operator} amdgpu_driver_version=${amdgpu_driver_version}"
}

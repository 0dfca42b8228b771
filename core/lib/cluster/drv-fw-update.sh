#!/usr/bin/env bash
# amdgpu kernel driver / GPU firmware update on the GPU nodes (replaces the Gaudi updater).
update_amdgpu_driver_firmware() {
    read_config_file || return 1
    echo "1) Driver only  2) Firmware only  3) Both"
    read -r -p "Select: " c
    local what
    case "$c" in 1) what=drivers ;; 2) what=firmware ;; 3) what=both ;; *) return 1 ;; esac
    execute_and_check "Updating amdgpu ${what}" ansible-playbook -i "${INVENTORY_PATH}" \
        playbooks/deploy-amdgpu-driver-firmware.yml \
        --extra-vars "update_target=${what} rocm_version=${rocm_version} amdgpu_driver_version=${amdgpu_driver_version}"
}

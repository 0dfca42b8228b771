#!/usr/bin/env bash
run_infrastructure_readiness_check() {
    [ "$skip_check" = "true" ] && { echo "Skipping infrastructure readiness checks"; return 0; }
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/inference-precheck.yml \
        --extra-vars "gpu_platform=${gpu_platform} cpu_or_gpu=${cpu_or_gpu}"
}

#!/usr/bin/env bash
run_istio_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-istio.yml 
}

#!/usr/bin/env bash
run_ingress_controller_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-ingress-controller.yml 
}

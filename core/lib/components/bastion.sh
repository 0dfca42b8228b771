#!/usr/bin/env bash
run_setup_bastion_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/setup-bastion.yml 
}

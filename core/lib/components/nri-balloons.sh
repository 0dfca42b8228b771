#!/usr/bin/env bash
deploy_nri_balloon_policy_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-cpu-optimization.yml --extra-vars cpu_playbook=true
}

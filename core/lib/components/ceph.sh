#!/usr/bin/env bash
run_deploy_ceph_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-ceph-storage.yml 
}

#!/usr/bin/env bash
# Rook-Ceph: render the cluster values from the inventory's storage nodes (hosts with a
# `devices:` list), then install the operator + cluster.
run_deploy_ceph_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/generate-ceph-values.yml || return 1
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-ceph-storage.yml
}

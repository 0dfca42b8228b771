#!/usr/bin/env bash
run_k8s_cluster_state_check() {
    ansible-playbook -i "${INVENTORY_PATH}" --become upgrade-cluster.yml --check
}
run_k8s_cluster_wait() {
    ansible kube_control_plane -i "${INVENTORY_PATH}" -m wait_for -a "port=6443 timeout=600"
}

#!/usr/bin/env bash
run_k8s_cluster_setup_kubeconfig() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/setup-user-kubeconfig.yml
}
run_label_nodes_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/label-nodes.yml \
        --extra-vars "cpu_or_gpu=${cpu_or_gpu} gpu_platform=${gpu_platform}"
}
run_deploy_cluster_config_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-cluster-config.yml \
        --extra-vars "secret_name=${cluster_url} cert_file=${cert_file} key_file=${key_file}"
}

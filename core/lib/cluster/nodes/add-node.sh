#!/usr/bin/env bash
add_worker_node() {
    read_config_file || return 1
    read -r -p "Name of the new worker node (as in hosts.yaml): " node
    [ -z "$node" ] && return 1
    execute_and_check "Preparing the environment" setup_initial_env
    execute_and_check "Adding node $node" ansible-playbook -i "${INVENTORY_PATH}" --become \
        --become-user=root scale.yml --limit="$node"
    execute_and_check "Labelling nodes" run_label_nodes_playbook
    if [ "$cpu_or_gpu" = "c" ] && [ "$deploy_nri_balloon_policy" = "yes" ]; then
        execute_and_check "Re-applying NRI balloons" deploy_nri_balloon_policy_playbook
    fi
}

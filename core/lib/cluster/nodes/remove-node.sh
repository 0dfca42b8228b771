#!/usr/bin/env bash
remove_worker_node() {
    read_config_file || return 1
    read -r -p "Name of the worker node to remove: " node
    [ -z "$node" ] && return 1
    execute_and_check "Preparing the environment" setup_initial_env
    execute_and_check "Removing node $node" ansible-playbook -i "${INVENTORY_PATH}" --become \
        --become-user=root remove-node.yml -e node="$node" -e skip_confirmation=yes
}

#!/usr/bin/env bash
install_kubernetes() {
    ansible-playbook -i "${INVENTORY_PATH}" cluster.yml --become --become-user=root
}

#!/usr/bin/env bash
run_reset_playbook() {
    if [ "$uninstall_ceph" = "yes" ]; then
        ansible-playbook -i "${INVENTORY_PATH}" playbooks/uninstall-ceph-storage.yml || return 1
    fi
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-keycloak-controller.yml \
        --extra-vars "delete_pv_on_purge=yes" || true
    ansible-playbook -i "${INVENTORY_PATH}" --become --become-user=root reset.yml \
        -e reset_confirmation=yes || return 1
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/reset.yml
}

reset_cluster() {
    read -r -p "This destroys the cluster and its data. Type 'yes' to continue: " ok
    [ "$ok" = "yes" ] || { echo "Aborted"; return 1; }
    execute_and_check "Preparing the environment" invoke_prereq_workflows
    execute_and_check "Purging the cluster" run_reset_playbook
}

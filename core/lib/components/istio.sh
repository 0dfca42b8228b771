#!/usr/bin/env bash
# Istio ambient mesh: upstream charts, or OpenShift Service Mesh 3 on OpenShift.
run_istio_playbook() {
    if [ "${kubernetes_platform:-vanilla}" = "openshift" ]; then
        KUBERNETES_PLATFORM=openshift ansible-playbook -i "${INVENTORY_PATH}" \
            playbooks/deploy-istio-openshift.yml --extra-vars "kubernetes_platform=openshift"
    else
        ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-istio.yml
    fi
}

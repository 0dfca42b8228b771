#!/usr/bin/env bash
# Deploy onto an existing cluster: import kubeconfig, detect the platform, localhost inventory.
manage_kubeconfig() {
    local kc="${KUBECONFIG:-$HOME/.kube/config}"
    if [ ! -f "$kc" ]; then
        read -r -p "Path to the kubeconfig of the existing cluster: " kc
    fi
    [ -f "$kc" ] || { echo "kubeconfig $kc not found" >&2; return 1; }
    mkdir -p "$HOME/.kube" && [ "$kc" != "$HOME/.kube/config" ] && cp "$kc" "$HOME/.kube/config"
    kubectl cluster-info >/dev/null || { echo "cluster not reachable" >&2; return 1; }
}

detect_kubernetes_platform() {
    if kubectl api-resources 2>/dev/null | grep -q "route.openshift.io"; then
        kubernetes_platform="openshift"
    elif kubectl get nodes -o jsonpath='{.items[0].spec.providerID}' 2>/dev/null | grep -q '^aws'; then
        kubernetes_platform="eks"
    elif kubectl get nodes -o jsonpath='{.items[0].spec.providerID}' 2>/dev/null | grep -q '^gce'; then
        kubernetes_platform="gke"
    elif kubectl get nodes -o jsonpath='{.items[0].spec.providerID}' 2>/dev/null | grep -q '^azure'; then
        kubernetes_platform="aks"
    else
        kubernetes_platform="vanilla"
    fi
    echo "Detected platform: $kubernetes_platform"
}

write_brownfield_inventory() {
    cat > "$brownfield_deployment_host_file" <<INV
all:
  hosts:
    localhost:
      ansible_connection: local
      ansible_python_interpreter: ${python3_interpreter:-/usr/bin/python3}
  children:
    kube_control_plane:
      hosts:
        localhost:
INV
}

brownfield_deployment() {
    brownfield_deployment="yes"
    manage_kubeconfig || return 1
    detect_kubernetes_platform
    write_brownfield_inventory
    INVENTORY_PATH=$brownfield_deployment_host_file
    fresh_installation
}

#!/usr/bin/env bash
# Enterprise inference stack on AMD Instinct MI355X: provision / decommission / update /
# brownfield deployment of Kubernetes + gateways + observability + the MI355X serving runtime.
#
#   ./inference-stack-deploy.sh [--cluster-url URL --cert-file F --key-file F
#        --keycloak-client-id ID --keycloak-admin-user U --keycloak-admin-password P
#        --hugging-face-token T --models 1,9 --cpu-or-gpu mi355x|cpu
#        --deploy-nri-balloon-policy yes|no --skip-check]
set -o pipefail

SCRIPT_DIR="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
CORE_DIR="$SCRIPT_DIR"

if [ -t 1 ] && command -v tput >/dev/null 2>&1; then
    RED=$(tput setaf 1); GREEN=$(tput setaf 2); YELLOW=$(tput setaf 3); BLUE=$(tput setaf 4)
    NC=$(tput sgr0)
else
    RED=""; GREEN=""; YELLOW=""; BLUE=""; NC=""
fi

for f in \
    lib/system/config-vars.sh lib/system/execute-and-check.sh lib/system/setup-env.sh \
    lib/system/precheck/read-config-file.sh lib/system/precheck/prereq-check.sh \
    lib/system/precheck/readiness-check.sh lib/user-menu/parse-user-prompts.sh \
    lib/user-menu/user-menu.sh lib/models/model-catalog.sh lib/models/model-selection.sh \
    lib/models/install-model.sh lib/models/install-model-hf.sh lib/models/uninstall-model.sh \
    lib/models/uninstall-model-hf.sh lib/models/list-model.sh \
    lib/cluster/deployment/fresh-install.sh lib/cluster/deployment/cluster-purge.sh \
    lib/cluster/deployment/cluster-update.sh lib/cluster/nodes/add-node.sh \
    lib/cluster/nodes/remove-node.sh lib/cluster/config/cluster-config.sh \
    lib/cluster/state/cluster-state-check.sh lib/cluster/drv-fw-update.sh \
    lib/components/kubernetes-setup.sh lib/components/ingress-controller.sh \
    lib/components/amd-gpu-operator.sh lib/components/keycloak.sh \
    lib/components/genai-gateway.sh lib/components/observability.sh lib/components/istio.sh \
    lib/components/ceph.sh lib/components/nri-balloons.sh lib/components/bastion.sh \
    lib/brownfield/brownfield_deployment.sh; do
    # shellcheck disable=SC1090
    source "$CORE_DIR/$f"
done

usage() {
    sed -n '2,9p' "${BASH_SOURCE[0]}" | sed 's/^# \{0,1\}//'
}

main_menu() {
    parse_arguments "$@"
    echo "${BLUE}Enterprise Inference on AMD Instinct MI355X${NC}"
    echo "1) Provision Enterprise Inference Cluster"
    echo "2) Decommission Existing Cluster"
    echo "3) Update Existing Cluster"
    echo "4) Brownfield Deployment (existing Kubernetes cluster)"
    read -r -p "Select an option: " choice
    case "$choice" in
        1) read -r -p "Provision a new cluster? (yes/no): " ok
           [ "$ok" = "yes" ] && fresh_installation ;;
        2) reset_cluster ;;
        3) update_cluster ;;
        4) brownfield_deployment ;;
        *) echo "${RED}Invalid option${NC}" >&2; exit 1 ;;
    esac
}

if [[ "${BASH_SOURCE[0]}" == "${0}" ]]; then
    main_menu "$@"
fi

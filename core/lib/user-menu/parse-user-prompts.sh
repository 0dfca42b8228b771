#!/usr/bin/env bash
# CLI flags (--cluster-url ... --skip-check) and prompts for anything still unset.
parse_arguments() {
    while [[ $# -gt 0 ]]; do
        case "$1" in
            --cluster-url) cluster_url="$2"; shift 2 ;;
            --cert-file) cert_file="$2"; shift 2 ;;
            --key-file) key_file="$2"; shift 2 ;;
            --keycloak-client-id) keycloak_client_id="$2"; shift 2 ;;
            --keycloak-admin-user) keycloak_admin_user="$2"; shift 2 ;;
            --keycloak-admin-password) keycloak_admin_password="$2"; shift 2 ;;
            --hugging-face-token) hugging_face_token="$2"; shift 2 ;;
            --models) models="$2"; shift 2 ;;
            --cpu-or-gpu) cpu_or_gpu="$2"; shift 2 ;;
            --deploy-nri-balloon-policy) deploy_nri_balloon_policy="$2"; shift 2 ;;
            --skip-check) skip_check="true"; shift ;;
            -h|--help) usage; exit 0 ;;
            *) echo "Unknown option: $1" >&2; usage; exit 1 ;;
        esac
    done
}

prompt_for_input() {
    [ -z "$cluster_url" ] && read -r -p "Enter the cluster URL (FQDN): " cluster_url
    [ -z "$cert_file" ] && read -r -p "Enter the full path to the TLS certificate file: " cert_file
    [ -z "$key_file" ] && read -r -p "Enter the full path to the TLS key file: " key_file
    if [ "$deploy_keycloak" = "yes" ]; then
        [ -z "$keycloak_client_id" ] && read -r -p "Enter the Keycloak client id: " keycloak_client_id
        [ -z "$keycloak_admin_user" ] && read -r -p "Enter the Keycloak admin user: " keycloak_admin_user
        [ -z "$keycloak_admin_password" ] && read -r -s -p "Enter the Keycloak admin password: " keycloak_admin_password && echo
    fi
    if [ -z "$cpu_or_gpu" ]; then
        read -r -p "Deploy on AMD Instinct GPUs or CPU? (mi355x/cpu): " cpu_or_gpu
        normalise_platform || return 1
    fi
    if [ "$cpu_or_gpu" = "c" ] && [ -z "$deploy_nri_balloon_policy" ]; then
        deploy_nri_balloon_policy="yes"   # CPU serving pins cores with NRI balloons
    fi
    for v in deploy_kubernetes_fresh deploy_ingress_controller deploy_keycloak deploy_genai_gateway \
             deploy_observability deploy_llm_models deploy_ceph deploy_istio; do
        if [ -z "${!v}" ]; then
            read -r -p "${v//_/ }? (yes/no): " ans
            printf -v "$v" '%s' "$ans"
        fi
    done
    [ "$deploy_keycloak" = "yes" ] && deploy_apisix="yes"
    model_selection
}

#!/usr/bin/env bash
# Provision: Kubernetes -> cluster config -> AMD GPU operator (or NRI balloons on CPU) -> storage
# -> ingress -> Keycloak/APISIX or GenAI gateway -> observability -> mesh -> models.
fresh_installation() {
    if [ "$brownfield_deployment" = "yes" ]; then
        deploy_kubernetes_fresh="no"
        skip_check="true"
    fi
    read_config_file || return 1
    prompt_for_input || return 1
    execute_and_check "Setting up the deployment environment" setup_initial_env
    cd "$KUBESPRAYDIR" || return 1
    if [ "$brownfield_deployment" = "yes" ]; then
        execute_and_check "Preparing the bastion host" run_setup_bastion_playbook
    fi
    if [ "$deploy_kubernetes_fresh" = "yes" ]; then
        execute_and_check "Installing Kubernetes" install_kubernetes
    fi
    execute_and_check "Applying cluster configuration" run_deploy_cluster_config_playbook
    if [ "$cpu_or_gpu" = "c" ] && [ "$deploy_nri_balloon_policy" = "yes" ]; then
        execute_and_check "Deploying NRI CPU balloon policy" deploy_nri_balloon_policy_playbook
    fi
    if [ "$cpu_or_gpu" = "g" ] && [ "$deploy_amd_gpu_operator" = "yes" ]; then
        execute_and_check "Deploying the AMD GPU Operator" run_deploy_amd_gpu_operator_playbook
    fi
    if [ "$deploy_ceph" = "yes" ]; then
        execute_and_check "Deploying Ceph storage" run_deploy_ceph_playbook
    fi
    if [ "$deploy_ingress_controller" = "yes" ]; then
        execute_and_check "Deploying the ingress controller" run_ingress_controller_playbook
    fi
    if [ "$deploy_keycloak" = "yes" ]; then
        execute_and_check "Deploying Keycloak + APISIX" run_keycloak_playbook
    fi
    if [ "$deploy_genai_gateway" = "yes" ]; then
        execute_and_check "Deploying the GenAI gateway" run_genai_gateway_playbook
    fi
    if [ "$deploy_observability" = "yes" ]; then
        execute_and_check "Deploying observability" run_observability_playbook
    fi
    if [ "$deploy_istio" = "yes" ]; then
        execute_and_check "Deploying Istio" run_istio_playbook
    fi
    if [ "$deploy_llm_models" = "yes" ]; then
        execute_and_check "Deploying inference models" deploy_inference_llm_models_playbook
    fi
    echo "${GREEN:-}Inference stack is up: https://${cluster_url}${NC:-}"
}

run_fresh_install_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" --become --become-user=root cluster.yml
}

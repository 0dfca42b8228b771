#!/usr/bin/env bash
# Build the Ansible tag list + extra-vars for the selected models and run the model playbook.
build_model_tags() {   # prefix (install|uninstall) -> "prefix-a,prefix-b[,install-genai-gateway]"
    local prefix=$1 tags="" m
    for m in $model_name_list; do
        tags+="${prefix}-${m},"
    done
    if [ -n "$huggingface_model_deployment_name" ]; then
        tags+="${prefix}-${huggingface_model_deployment_name},"
    fi
    if [ "$prefix" = "install" ]; then
        [ "$deploy_keycloak" = "yes" ] && tags+="install-keycloak-apisix,"
        [ "$deploy_genai_gateway" = "yes" ] && tags+="install-genai-gateway,"
    fi
    echo "${tags%,}"
}

model_extra_vars() {
    local values_file="$mi355x_values_file_path"
    [ "$cpu_or_gpu" = "c" ] && values_file="$xeon_values_file_path"
    local apisix_enabled="false" ingress_enabled="false" metrics="false"
    [ "$deploy_apisix" = "yes" ] && apisix_enabled="true"
    [ "$deploy_keycloak" = "yes" ] && ingress_enabled="true"
    [ "$deploy_observability" = "yes" ] && metrics="true"
    echo "kubernetes_platform=${kubernetes_platform} secret_name=${cluster_url} cert_file=${cert_file}" \
         "key_file=${key_file} keycloak_admin_user=${keycloak_admin_user}" \
         "keycloak_admin_password=${keycloak_admin_password} keycloak_client_id=${keycloak_client_id}" \
         "hugging_face_token=${hugging_face_token} model_name_list='${model_name_list// /,}'" \
         "cpu_or_gpu=${cpu_or_gpu} gpu_platform=${gpu_platform} platform_values_file=${values_file}" \
         "apisix_enabled=${apisix_enabled} ingress_enabled=${ingress_enabled}" \
         "deploy_keycloak=${deploy_keycloak} deploy_genai_gateway=${deploy_genai_gateway}" \
         "vllm_metrics_enabled=${metrics} deploy_ceph=${deploy_ceph}" \
         "huggingface_model_id=${huggingface_model_id} runtime_image=${runtime_image:-}" \
         "huggingface_model_deployment_name=${huggingface_model_deployment_name}" \
         "huggingface_tensor_parellel_size=${huggingface_tensor_parellel_size}"
}

deploy_inference_llm_models_playbook() {
    local tags
    tags=$(build_model_tags install)
    [ "$brownfield_deployment" = "yes" ] && INVENTORY_PATH=$brownfield_deployment_host_file
    echo "Deploying models with tags: $tags"
    # shellcheck disable=SC2046
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-inference-models.yml \
        --extra-vars "$(model_extra_vars) install_true=true" --tags "$tags" \
        --vault-password-file "$vault_pass_file"
}

add_model() {
    read_config_file || return 1
    deploy_llm_models="yes"
    model_selection || return 1
    execute_and_check "Deploying inference models" deploy_inference_llm_models_playbook
}

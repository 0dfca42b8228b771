#!/usr/bin/env bash
remove_model_deployed_via_huggingface() {
    read -r -p "Enter the deployment (release) name to remove: " huggingface_model_deployment_name
    [ -z "$huggingface_model_deployment_name" ] && { echo "No name given" >&2; return 1; }
    model_name_list=""
    execute_and_check "Removing ${huggingface_model_deployment_name}" remove_inference_llm_models_playbook
}

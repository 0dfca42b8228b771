#!/usr/bin/env bash
# Deploy any Hugging Face model id as a custom release (vllm chart + mi355x values).
deploy_from_huggingface() {
    read -r -p "Enter the Hugging Face model id (e.g. org/model): " huggingface_model_id
    read -r -p "Enter a deployment (release) name: " huggingface_model_deployment_name
    read -r -p "Enter the tensor parallel size (1-8): " huggingface_tensor_parellel_size
    if ! [[ "$huggingface_tensor_parellel_size" =~ ^[1-8]$ ]]; then
        echo "Tensor parallel size must be an integer in 1..8" >&2
        return 1
    fi
    if ! [[ "$huggingface_model_deployment_name" =~ ^[a-z0-9]([-a-z0-9]*[a-z0-9])?$ ]]; then
        echo "Deployment name must be a DNS-1123 label" >&2
        return 1
    fi
    hugging_face_model_deployment="true"
    deploy_llm_models="yes"
    model_name_list=""
    execute_and_check "Deploying ${huggingface_model_id}" deploy_inference_llm_models_playbook
}

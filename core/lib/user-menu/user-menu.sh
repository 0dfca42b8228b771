#!/usr/bin/env bash
manage_worker_nodes() {
    echo "1) Add worker node"
    echo "2) Remove worker node"
    read -r -p "Select: " c
    case "$c" in
        1) add_worker_node ;;
        2) remove_worker_node ;;
        *) echo "Invalid choice" >&2; return 1 ;;
    esac
}

manage_models() {
    echo "1) Add model(s) from the catalog"
    echo "2) Remove model(s)"
    echo "3) List deployed models"
    echo "4) Deploy a model from Hugging Face"
    echo "5) Remove a Hugging Face model deployment"
    read -r -p "Select: " c
    case "$c" in
        1) add_model ;;
        2) remove_model ;;
        3) read_config_file && list_inference_llm_models_playbook ;;
        4) read_config_file && deploy_from_huggingface ;;
        5) read_config_file && remove_model_deployed_via_huggingface ;;
        *) echo "Invalid choice" >&2; return 1 ;;
    esac
}

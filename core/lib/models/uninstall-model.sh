#!/usr/bin/env bash
remove_inference_llm_models_playbook() {
    local tags
    tags=$(build_model_tags uninstall)
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-inference-models.yml \
        --extra-vars "$(model_extra_vars) install_true=false" --tags "$tags" \
        --vault-password-file "$vault_pass_file"
}

remove_model() {
    read_config_file || return 1
    deploy_llm_models="yes"
    model_selection || return 1
    execute_and_check "Removing inference models" remove_inference_llm_models_playbook
}

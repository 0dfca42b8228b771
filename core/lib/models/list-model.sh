#!/usr/bin/env bash
list_inference_llm_models_playbook() {
    ansible-playbook -i "${INVENTORY_PATH}" playbooks/deploy-inference-models.yml --tags list-models
}

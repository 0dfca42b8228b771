#!/usr/bin/env bash
# Interactive / scripted model selection: numbers (GPU 1-14, CPU 21-26) -> canonical names.
model_selection() {
    if [ "${list_model_menu:-}" = "skip" ]; then
        return 0
    fi
    if [ -z "$hugging_face_token" ] && [ "$deploy_llm_models" = "yes" ]; then
        read -r -p "Enter the token for Huggingface: " hugging_face_token
    fi
    if [ -z "$deploy_llm_models" ]; then
        read -r -p "Do you want to proceed with deploying Large Language Model (LLM)? (yes/no): " deploy_llm_models
    fi
    [ "$deploy_llm_models" = "yes" ] || return 0
    [ "$hugging_face_model_deployment" = "true" ] && return 0
    if [ -z "$models" ]; then
        local plat="gpu"
        [ "$cpu_or_gpu" = "c" ] && plat="cpu"
        echo "Available models for ${plat^^} deployment:"
        print_model_menu "$plat"
        read -r -p "Enter the numbers of the models to deploy/remove (comma-separated, e.g. 1,3,5): " models
    fi
    model_name_list=$(get_model_names) || return 1
    echo "Selected models: $model_name_list"
}

# "1,9" -> "llama-8b mixtral-8x-7b"; rejects GPU numbers on CPU and vice versa.
get_model_names() {
    local names=() m name plat
    IFS=',' read -ra picked <<< "$models"
    for m in "${picked[@]}"; do
        m="${m//[[:space:]]/}"
        [ -z "$m" ] && continue
        if ! [[ "$m" =~ ^[0-9]+$ ]]; then
            echo "Error: invalid model selection '$m'" >&2
            return 1
        fi
        name=$(catalog_field "$m" 2)
        plat=$(catalog_field "$m" 8)
        if [ -z "$name" ]; then
            echo "Error: unknown model number $m" >&2
            return 1
        fi
        if [ "$cpu_or_gpu" = "c" ] && [ "$plat" != "cpu" ]; then
            echo "Error: GPU model identifier $m provided for CPU deployment/removal." >&2
            return 1
        fi
        if [ "$cpu_or_gpu" = "g" ] && [ "$plat" != "gpu" ]; then
            echo "Error: CPU model identifier $m provided for GPU deployment/removal." >&2
            return 1
        fi
        names+=("$name")
    done
    echo "${names[*]}"
}

#!/usr/bin/env bash
# Parse inference-config.cfg (+ metadata pins).  on/off -> yes/no, platform normalisation,
# gateway mode exclusivity.  Values already given on the command line win over the file.
_cfg_set() {   # key value: only when not set by a CLI flag
    local k=$1 v=$2
    if [ -z "${!k:-}" ] || [ "${cfg_file_overrides_cli:-false}" = "true" ]; then
        printf -v "$k" '%s' "$v"
    fi
}

read_config_file() {
    local file="${1:-$inference_config_file}"
    if [ ! -f "$file" ]; then
        echo "Configuration file $file not found" >&2
        return 1
    fi
    while IFS='=' read -r key value || [ -n "$key" ]; do
        key="${key//[[:space:]]/}"
        [[ -z "$key" || "$key" == \#* ]] && continue
        value="${value%%#*}"
        value="$(echo "$value" | sed -e 's/^[[:space:]]*//' -e 's/[[:space:]]*$//' -e 's/^"//' -e 's/"$//')"
        case "$value" in
            on) value="yes" ;;
            off) value="no" ;;
        esac
        case "$key" in
            deploy_keycloak_apisix) _cfg_set deploy_keycloak "$value"; _cfg_set deploy_apisix "$value" ;;
            *) _cfg_set "$key" "$value" ;;
        esac
    done < "$file"
    if [ -f "$metadata_config_file" ]; then
        while IFS='=' read -r key value || [ -n "$key" ]; do
            key="${key//[[:space:]]/}"
            [[ -z "$key" || "$key" == \#* ]] && continue
            value="${value%\"}"; value="${value#\"}"
            printf -v "$key" '%s' "$value"
        done < "$metadata_config_file"
    fi
    normalise_platform || return 1
    if [ "${deploy_genai_gateway:-no}" = "yes" ] && [ "${deploy_keycloak:-no}" = "yes" ]; then
        echo "GenAI gateway and Keycloak/APISIX are mutually exclusive; enable only one." >&2
        return 1
    fi
    if [ -n "${vault_pass_code:-}" ]; then
        umask 077
        printf '%s' "$vault_pass_code" > "$vault_pass_file"
    fi
    if [ -n "${http_proxy:-}" ] && [ -f "${KUBESPRAYDIR}/inventory/mycluster/group_vars/all/all.yml" ]; then
        sed -i -e "s|^# *http_proxy:.*|http_proxy: \"$http_proxy\"|" \
               -e "s|^# *https_proxy:.*|https_proxy: \"${https_proxy:-$http_proxy}\"|" \
               -e "s|^# *no_proxy:.*|no_proxy: \"${no_proxy:-}\"|" \
               "${KUBESPRAYDIR}/inventory/mycluster/group_vars/all/all.yml"
    fi
    return 0
}

# cpu_or_gpu: c|cpu -> c ; g|gpu|amd|mi355x|mi300x -> g (AMD GPU Operator path)
normalise_platform() {
    case "${cpu_or_gpu,,}" in
        c|cpu|xeon|epyc) cpu_or_gpu="c"; gpu_platform="cpu"; deploy_amd_gpu_operator="no" ;;
        g|gpu|amd) cpu_or_gpu="g"; gpu_platform="${gpu_platform:-mi355x}"; deploy_amd_gpu_operator="${deploy_amd_gpu_operator:-yes}" ;;
        mi355x) cpu_or_gpu="g"; gpu_platform="mi355x"; deploy_amd_gpu_operator="${deploy_amd_gpu_operator:-yes}" ;;
        mi300x|mi325x) gpu_platform="${cpu_or_gpu,,}"; cpu_or_gpu="g"; deploy_amd_gpu_operator="${deploy_amd_gpu_operator:-yes}" ;;
        gaudi2|gaudi3)
            echo "cpu_or_gpu=${cpu_or_gpu}: Intel Gaudi is not supported by this stack; use mi355x" >&2
            return 1 ;;
        "") ;;
        *) echo "Unknown cpu_or_gpu value '${cpu_or_gpu}' (use cpu or mi355x)" >&2; return 1 ;;
    esac
    return 0
}

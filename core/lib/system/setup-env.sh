#!/usr/bin/env bash
# Deploy-node bootstrap: Kubespray checkout, Python venv, copy charts/playbooks/roles/inventory
# into the Kubespray tree, vault secrets, Ansible collections.
setup_initial_env() {
    run_system_prerequisites_check || return 1
    if [ ! -d "$KUBESPRAYDIR" ]; then
        git clone https://github.com/kubernetes-sigs/kubespray.git "$KUBESPRAYDIR" || return 1
    fi
    (cd "$KUBESPRAYDIR" && git fetch --tags -q && git checkout -q "${kubespray_version:-v2.27.0}") || return 1
    if [ ! -d "$VENVDIR" ]; then
        python3 -m venv "$VENVDIR" || return 1
    fi
    # shellcheck disable=SC1091
    source "$VENVDIR/bin/activate"
    pip install -q -U pip && pip install -q -r "$KUBESPRAYDIR/requirements.txt" kubernetes || return 1
    mkdir -p "$KUBESPRAYDIR/inventory/mycluster"
    if [ ! -d "$KUBESPRAYDIR/inventory/mycluster/group_vars" ]; then
        cp -r "$KUBESPRAYDIR/inventory/sample/." "$KUBESPRAYDIR/inventory/mycluster/"
    fi
    cp "$CORE_DIR/inventory/hosts.yaml" "$KUBESPRAYDIR/inventory/mycluster/hosts.yaml"
    cp "$CORE_DIR/inventory/metadata/all.yml" "$KUBESPRAYDIR/inventory/mycluster/group_vars/all/all.yml"
    cp "$CORE_DIR/inventory/metadata/addons.yml" "$KUBESPRAYDIR/inventory/mycluster/group_vars/k8s_cluster/addons.yml"
    for d in playbooks roles helm-charts scripts; do
        cp -r "$CORE_DIR/$d" "$KUBESPRAYDIR/"
    done
    mkdir -p "$KUBESPRAYDIR/config/vars"
    cp "$CORE_DIR"/inventory/metadata/vars/*.yml "$KUBESPRAYDIR/config/vars/"
    local vault="$KUBESPRAYDIR/config/vault.yml"
    # the reference's mandatory keys (its setup-env.sh:108-129) plus this stack's additions
    local required=(litellm_master_key litellm_salt_key redis_password langfuse_secret_key \
                    langfuse_public_key postgresql_username postgresql_password \
                    clickhouse_username clickhouse_password langfuse_login langfuse_user \
                    langfuse_password minio_secret minio_user postgres_user postgres_password \
                    grafana_admin_password langfuse_salt langfuse_nextauth_secret \
                    langfuse_encryption_key valkey_password keycloak_db_password)
    local regenerate=false
    for k in "${required[@]}"; do
        grep -q "^${k}:" "$vault" 2>/dev/null || regenerate=true
    done
    if [ "$regenerate" = true ]; then
        bash "$CORE_DIR/scripts/generate-vault-secrets.sh" "$vault" || return 1
    fi
    ansible-galaxy collection install -q kubernetes.core community.general || return 1
    cd "$KUBESPRAYDIR" || return 1
    run_infrastructure_readiness_check
}

invoke_prereq_workflows() {
    read_config_file || return 1
    setup_initial_env
}

#!/usr/bin/env bash
# Generate random secrets for the gateway / tracing / monitoring stacks into an Ansible vault
# variables file (mode 0600).  Usage: generate-vault-secrets.sh <vault.yml>
set -euo pipefail
out="${1:-config/vault.yml}"
mkdir -p "$(dirname "$out")"
rand() { openssl rand -hex "${1:-24}"; }
umask 077
cat > "$out" <<YML
litellm_master_key: "sk-$(rand 24)"
litellm_salt_key: "sk-$(rand 24)"
redis_password: "$(rand 16)"
langfuse_secret_key: "sk-lf-$(rand 16)"
langfuse_public_key: "pk-lf-$(rand 16)"
langfuse_salt: "$(rand 16)"
langfuse_nextauth_secret: "$(rand 24)"
langfuse_encryption_key: "$(rand 32)"
postgresql_username: "litellm"
postgresql_password: "$(rand 16)"
langfuse_postgresql_password: "$(rand 16)"
clickhouse_password: "$(rand 16)"
minio_user: "minio"
minio_secret: "$(rand 16)"
valkey_password: "$(rand 16)"
grafana_admin_password: "$(rand 12)"
keycloak_db_password: "$(rand 16)"
YML
chmod 600 "$out"
echo "wrote $out"

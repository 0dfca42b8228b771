#!/usr/bin/env bash
# Generate random secrets for the gateway / tracing / monitoring stacks into the Ansible
# variables file every secret-consuming play loads (vars_files: ../config/vault.yml).
# Key names are those of the reference's vault (core/scripts/generate-vault-secrets.sh there),
# so an existing vault.yml keeps working; the extra keys at the end are MI355X-stack additions.
# Usage: generate-vault-secrets.sh <vault.yml>
set -euo pipefail
out="${1:-config/vault.yml}"
mkdir -p "$(dirname "$out")"
hex() { openssl rand -hex "${1:-16}"; }
# alphanumeric (URL/DSN safe)
pw() { openssl rand -base64 48 | tr -dc 'A-Za-z0-9' | head -c "${1:-20}"; }
umask 077
cat > "$out" <<YML
# Auto-generated secrets (mode 0600) -- keep out of version control
litellm_master_key: "sk-$(hex 10)"
litellm_salt_key: "$(hex 10)"
redis_password: "$(pw 20)"
langfuse_secret_key: "lf_sk_$(hex 10)"
langfuse_public_key: "lf_pk_$(hex 10)"
postgresql_username: "admin"
postgresql_password: "$(pw 20)"
clickhouse_username: "default"
clickhouse_password: "$(pw 20)"
langfuse_login: "admin@admin.com"
langfuse_user: "admin"
langfuse_password: "Admin$(pw 20)!"
minio_secret: "$(pw 20)"
minio_user: "minio"
postgres_user: "postgres"
postgres_password: "$(pw 20)"
grafana_admin_password: "$(pw 20)"
langfuse_salt: "$(hex 16)"
langfuse_nextauth_secret: "$(hex 24)"
langfuse_encryption_key: "$(hex 32)"
valkey_password: "$(pw 20)"
keycloak_db_password: "$(pw 20)"
YML
chmod 600 "$out"
echo "wrote $out"

#!/usr/bin/env bash
# Create (or reuse) a confidential client with service accounts in the Keycloak realm and
# print its secret ("Client secret: ...") for the APISIX openid-connect plugin.
# Usage: keycloak-realmcreation.sh <keycloak_url> <admin_user> <admin_password> <client_id> [realm]
set -euo pipefail
KC_URL=$1; ADMIN=$2; PASS=$3; CLIENT=$4; REALM=${5:-master}
token=$(curl -sf -X POST "$KC_URL/realms/master/protocol/openid-connect/token" \
  -d grant_type=password -d client_id=admin-cli -d "username=$ADMIN" -d "password=$PASS" \
  | python3 -c 'import json,sys; print(json.load(sys.stdin)["access_token"])')
auth=(-H "Authorization: Bearer $token" -H "Content-Type: application/json")
existing=$(curl -sf "${auth[@]}" "$KC_URL/admin/realms/$REALM/clients?clientId=$CLIENT" \
  | python3 -c 'import json,sys; c=json.load(sys.stdin); print(c[0]["id"] if c else "")')
if [ -z "$existing" ]; then
  curl -sf "${auth[@]}" -X POST "$KC_URL/admin/realms/$REALM/clients" -d "{
    \"clientId\": \"$CLIENT\", \"enabled\": true, \"publicClient\": false,
    \"serviceAccountsEnabled\": true, \"standardFlowEnabled\": false,
    \"directAccessGrantsEnabled\": true, \"protocol\": \"openid-connect\",
    \"attributes\": {\"access.token.lifespan\": \"900\"}}"
  existing=$(curl -sf "${auth[@]}" "$KC_URL/admin/realms/$REALM/clients?clientId=$CLIENT" \
    | python3 -c 'import json,sys; print(json.load(sys.stdin)[0]["id"])')
fi
secret=$(curl -sf "${auth[@]}" "$KC_URL/admin/realms/$REALM/clients/$existing/client-secret" \
  | python3 -c 'import json,sys; print(json.load(sys.stdin)["value"])')
echo "Client secret: $secret"

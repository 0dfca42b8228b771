#!/usr/bin/env bash
# Print the secret of an existing Keycloak client.  Usage: <https://cluster_url> <admin> <pass> <client_id>
set -euo pipefail
BASE=$1; ADMIN=$2; PASS=$3; CLIENT=$4
token=$(curl -skf -X POST "$BASE/realms/master/protocol/openid-connect/token" \
  -d grant_type=password -d client_id=admin-cli -d "username=$ADMIN" -d "password=$PASS" \
  | python3 -c 'import json,sys; print(json.load(sys.stdin)["access_token"])')
id=$(curl -skf -H "Authorization: Bearer $token" "$BASE/admin/realms/master/clients?clientId=$CLIENT" \
  | python3 -c 'import json,sys; print(json.load(sys.stdin)[0]["id"])')
curl -skf -H "Authorization: Bearer $token" "$BASE/admin/realms/master/clients/$id/client-secret" \
  | python3 -c 'import json,sys; print(json.load(sys.stdin)["value"])'

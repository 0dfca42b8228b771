#!/usr/bin/env bash
# Menu number <-> canonical name <-> HF id, read from inventory/metadata/vars/model_catalog.yml
# (single source of truth shared with the Ansible model playbook).
_catalog_rows() {   # prints "number name model_id release chart tp mode platform"
    python3 - "$model_catalog_file" <<'PY'
import sys, yaml
for m in yaml.safe_load(open(sys.argv[1]))["model_catalog"]:
    print(m["number"], m["name"], m["model_id"], m["release"], m["chart"],
          m["tensor_parallel_size"], m["mode"], m["platform"])
PY
}

catalog_field() {   # catalog_field <number|name> <column 1-8>
    _catalog_rows | awk -v k="$1" -v c="$2" '$1 == k || $2 == k { print $c; exit }'
}

print_model_menu() {   # gpu|cpu
    local plat=$1
    _catalog_rows | awk -v p="$plat" '$8 == p { printf "%s. %s\n", $1, $3 }'
}

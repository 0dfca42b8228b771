#!/usr/bin/env bash
update_cluster() {
    echo "1) Manage worker nodes"
    echo "2) Manage LLM models"
    echo "3) Update AMD GPU driver / firmware"
    read -r -p "Select: " c
    case "$c" in
        1) manage_worker_nodes ;;
        2) manage_models ;;
        3) update_amdgpu_driver_firmware ;;
        *) echo "Invalid choice" >&2; return 1 ;;
    esac
}

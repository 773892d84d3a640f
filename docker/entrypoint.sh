#!/bin/bash
# Dispatch by first argument; default: run the given command.
set -e
case "${1:-}" in
  scheduler)     shift; exec python3 -m k8s_vgpu_scheduler_amd.cmd.scheduler "$@" ;;
  device-plugin) shift; /usr/local/bin/vgpu-init.sh "${HOOK_PATH:-/usr/local/vgpu}"
                 exec python3 -m k8s_vgpu_scheduler_amd.cmd.device_plugin "$@" ;;
  monitor)       shift; exec python3 -m k8s_vgpu_scheduler_amd.cmd.monitor "$@" ;;
  *)             exec "$@" ;;
esac

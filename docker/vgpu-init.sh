#!/bin/bash
# Install libmivgpu.so under the host hook path and (re)write ld.so.preload.
# Same contract as the device plugin's install step (cmd/device_plugin.py
# install_shim): <dest>/libmivgpu.so, <dest>/ld.so.preload, <dest>/containers/.
# The copy is atomic (tmp + rename) so running containers keep a valid mapping.
set -euo pipefail
DEST_DIR=${1:-${HOOK_PATH:-/usr/local/vgpu}}
SRC=${MIVGPU_LIB:-/opt/mivgpu/k8s_vgpu_scheduler_amd/lib/libmivgpu.so}
CONTAINER_LIB=/usr/local/vgpu/libmivgpu.so

if [ ! -f "$SRC" ]; then
  echo "vgpu-init: $SRC not found" >&2
  exit 1
fi
mkdir -p "$DEST_DIR/containers"
if ! cmp -s "$SRC" "$DEST_DIR/libmivgpu.so"; then
  cp "$SRC" "$DEST_DIR/libmivgpu.so.tmp"
  mv -f "$DEST_DIR/libmivgpu.so.tmp" "$DEST_DIR/libmivgpu.so"
  echo "vgpu-init: installed $DEST_DIR/libmivgpu.so"
fi
echo "$CONTAINER_LIB" > "$DEST_DIR/ld.so.preload.tmp"
mv -f "$DEST_DIR/ld.so.preload.tmp" "$DEST_DIR/ld.so.preload"

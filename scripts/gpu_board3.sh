set -o pipefail
out=gpurun_out/board3; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_shim_gpu.py -x -v -s --timeout 300 --timeout-method thread -k "governor" > $out/tests.log 2>&1 || exit 1
ls -la /tmp/vgpulock > $out/lockdir.txt 2>&1
python -c "
from k8s_vgpu_scheduler_amd.smi import detect
from k8s_vgpu_scheduler_amd.monitor import board
be = detect(None)
for g in be.gpus():
    p = board.board_path(g.bdf)
    print(g.index, g.bdf, p, p.exists() if p else None, board.read_slots(p)[:3] if p else None)
" > $out/board_map.txt 2>&1 || true

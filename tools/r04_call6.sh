# round 4: batching with per-connection arenas, receive side, hooks under load
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u tools/batch_arena_sweep.py > gpurun_out/r04/batch_arena_sweep.log 2>&1

# N1: the DFA walks' share of C4 (ablation bound for any LDS staging of rule DFAs); 2-rank rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3n1; mkdir -p $o
timeout -k 10 300 python tools/steady.py c4 "" MXP_DEBUG_FLAGS=16777216 > $o/steady_c4_nodfa.log 2>&1 || exit $?
MXP_REHEARSE_MULTI=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $o/rehearse2.log 2>&1 || exit $?

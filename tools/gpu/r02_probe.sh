#!/bin/bash
# Round-2 first call: host CPU facts for cpu_baseline, the GPU suite, one bench line.
set -o pipefail
OUT=gpurun_out/r02_probe
mkdir -p $OUT
export TMPDIR=/tmp
{ lscpu; echo; nproc; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; env | grep -E 'OMP|MAX_JOBS'; } > $OUT/cpu.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_cog.json 2> $OUT/bench_cog.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_cog.json

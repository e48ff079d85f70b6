set -o pipefail
O=gpurun_out/r05_c6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag/pred_trace.py cog pred ptrace > $O/trace_base.log 2>&1 && \
timeout -k 10 200 python tools/diag/pred_trace.py cog pred q2trace > $O/trace_q2.log 2>&1 && \
timeout -k 10 200 python tools/diag/pred_trace.py cog pred l3trace > $O/trace_l3.log 2>&1 && \
timeout -k 10 200 python tools/diag/pred_stamps.py cog pred > $O/stamps_cog_pred.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/pmc1 -o run -- python3 tools/attn_only.py cog 3 pred > $O/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc2 -o run -- python3 tools/attn_only.py cog 3 pred > $O/pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum --output-format csv -d $O/pmc3 -o run -- python3 tools/attn_only.py cog 3 pred > $O/pmc3.log 2>&1
rc=$?
cat $O/trace*.log $O/stamps*.log | grep -v amdgpu.ids
python3 tools/pmc_summary.py $O mask_predict 2>&1 | head -30
tail -2 $O/pmc*.log
exit $rc

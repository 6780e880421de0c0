set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 tools/probes/store_probe 64 > $O/probe.txt 2>&1 || exit 1
cat $O/probe.txt
timeout -s KILL 60 rocprofv3 --pmc TCC_WRITE_sum TCC_NORMAL_WRITEBACK_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -T --output-format csv -d $O/p1 -o run -- tools/probes/store_probe 64 > $O/p1.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_STREAMING_REQ_sum -T --output-format csv -d $O/p2 -o run -- tools/probes/store_probe 64 > $O/p2.txt 2>&1 || exit 1
echo PROBE_DONE

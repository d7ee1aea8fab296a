cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 bash scripts/var_bench.sh c2:base c2:q64 c2:q66 c2:base c2:q64 c2:q66 || exit 1
SQ_GROUPS="3 2" timeout -k 10 400 bash scripts/sqprof.sh lds c2

# round 3: where k_lzscan / k_lzcand / k_search spend their cycles (natural 8192^2 -s1, one encode),
# two SQ counter passes; plus the +1-ulp chain parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_search.py -x -q --timeout 170 --timeout-method thread > gpurun_out/t7.log 2>&1 || { tail -20 gpurun_out/t7.log; exit 1; }
tail -2 gpurun_out/t7.log
timeout -k 10 150 python -u tools/scripts/natural_prof.py 8192 1 2 2>&1 | grep natural
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_s1a -o p -- python3 tools/scripts/natural_prof.py 8192 1 1 > gpurun_out/pmc_s1a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmc_s1b -o p -- python3 tools/scripts/natural_prof.py 8192 1 1 > gpurun_out/pmc_s1b.log 2>&1 || exit 1
ls gpurun_out/pmc_s1a gpurun_out/pmc_s1b

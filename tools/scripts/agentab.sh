set -e
mkdir -p gpurun_out/agentab
T=gpurun_out/agentab
HOH_LIB=var/agentmap.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests_agent.log 2>&1
tail -2 $T/tests_agent.log
for lib in hoh-ans_amd/lib/libhohgpu.so var/agentmap.so; do
  echo "== $lib"
  for sp in 2 3 4; do HOH_LIB=$lib timeout -k 10 120 python -u tools/scripts/natural_prof.py 8192 $sp 8; done
  HOH_LIB=$lib REPS=20 timeout -k 10 300 python -u tools/scripts/rep_speed.py 2 3 4
done

mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 900 python -m pytest tests -q -m "gpu"  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc2=$?
  echo "pytest rc=$rc2"; tail -30 gpurun_out/pytest_gpu.log
fi

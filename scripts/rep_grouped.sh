mkdir -p gpurun_out/r4o
export FMX_DEBUG=1
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  timeout -k 10 120 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 60 --timeout-method thread -k "every_layout_grouped and 4-2" > gpurun_out/r4o/rep_$i.log 2>&1
  rc=$?
  echo "rep $i rc=$rc $(tail -n 1 gpurun_out/r4o/rep_$i.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for i in 1 2 3; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_grouped.py -x -q --timeout 60 --timeout-method thread > gpurun_out/r4o/full_$i.log 2>&1
  rc=$?
  echo "full $i rc=$rc $(tail -n 1 gpurun_out/r4o/full_$i.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done

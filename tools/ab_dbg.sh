for dbg in 0 1 2 3; do
  SG_DBG=$dbg timeout -k 10 200 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 150 --timeout-method thread -k "c2_solve_matches" 2>&1 | tail -1 | sed "s/^/dbg=$dbg /"
done

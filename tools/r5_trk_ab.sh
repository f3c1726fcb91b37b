#!/bin/bash
# Timing-only tracker A/B: the front-end bench (C3 tracker us/frame) on variant libraries (tools/build_variant.sh)
# beside the default.  Usage: tools/r5_trk_ab.sh TAG name1 name2 ...  ("base" = the default library)
set -o pipefail
tag=${1:?tag}; shift
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=slam-robot_amd/csrc/libslamgpu_$v.so; fi
  SG_LIB_PATH=$lib timeout -k 10 200 python bench.py --only frontend --steps 20 --warmup 5 > gpurun_out/trkab_${tag}_$v.json 2>/dev/null || exit $?
  python - gpurun_out/trkab_${tag}_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["result"]["tracker"]
print("%-10s tracker %.1f us/frame, longest %d its" % (sys.argv[2], d["ms_per_frame_tracking"] * 1e3, d["newton_iterations_max_track"]))
PY
done

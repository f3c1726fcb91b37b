#!/bin/bash
# Phase-removal timing of the scaled sweep (SG_DBG bits: 1 no J store, 2 no point pass, 4 no camera pass,
# 8 no projection math).  Results are not valid linearizations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for f in ${DBG_LIST:-0 1 2 4 8 15}; do
  echo -n "SG_DBG=$f: "
  SG_DBG=$f timeout -k 10 100 python tools/sweep_only.py ${SWEEP_OBS:-2000000} 10 || break
done

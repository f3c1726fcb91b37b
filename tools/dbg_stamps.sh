for f in 0 1 2 8 11; do echo "SG_DBG=$f"; SG_DBG=$f timeout -k 10 60 python tools/stamp_check.py C2 | tail -9; done

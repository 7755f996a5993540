#!/bin/bash
# Diagnostic builds of the fp32 window kernel (ab/_C_p{0,1,2}.so: full / no network / no HBM stream),
# kernel alone on one 512-instance c3 range, alternating.
set -u
for rep in 1 2; do
  for v in 0 1 2; do
    cp ab/_C_p$v.so svoc/_C.so
    PROBE_TAG=$v timeout -k 10 120 python tools/winf_probe.py 512 10 || exit 1
  done
done
cp ab/_C_p0.so svoc/_C.so

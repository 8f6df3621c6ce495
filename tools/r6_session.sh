#!/bin/bash
# round-6 session: world-1 cost of the real RCCL paths (ProcessGroupNCCL vs the native communicator), replicated and
# sharded optimizer, and the modelled 8-rank step, final r6 tree
set -e
out=gpurun_out/r6d16
mkdir -p $out
timeout -k 10 1100 python tools/comm_pressure.py --rounds 2 --steps 60 --wgs 16 --cases torch,native,zero_torch,zero_native,dpnone,zero_dpnone,proxy_w16,zero_proxy_w16 > $out/comm_pressure.txt 2>&1
tail -9 $out/comm_pressure.txt

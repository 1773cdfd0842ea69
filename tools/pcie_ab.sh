#!/bin/bash
# A/B of the host-buffer (PCIe-inclusive) leg between two library builds.
O=gpurun_out/pcie_ab.txt
: > $O
for L in head default head default head default; do
  if [ $L = default ]; then LIB=""; else LIB=$PWD/tools/variants/libyta_$L.so; fi
  YTA_LIBRARY=$LIB timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/e2.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/e2.json').read().strip().splitlines()[-1])
print('$L', round(d['value']), 'pcie', round(d['pcie_inclusive']['value']), round(d['pcie_inclusive']['ms_per_step'],2))" >> $O
done
nproc >> $O; cat /sys/fs/cgroup/cpu.max >> $O 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O
cat $O

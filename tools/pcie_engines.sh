# GPU box: the host-buffer (PCIe-inclusive) leg of bench.py with 1 / 2 / 4 engines on as many host
# threads, pageable and page-locked caller buffers -> gpurun_out/pcie_ab.txt
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
: > $R/gpurun_out/pcie_ab.txt
for E in 1 2 4; do
  timeout -k 10 400 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-isolated --pcie-engines $E > $R/gpurun_out/pcie_$E.json 2>$R/gpurun_out/pcie_$E.err || { tail -3 $R/gpurun_out/pcie_$E.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/pcie_$E.json').read().strip().splitlines()[-1]); p=d['pcie_inclusive']; q=p['pinned']
print('pcie engines $E pageable', round(p['value']), 'ms %.2f' % p['ms_per_step'], '| pinned', round(q['value']), 'ms %.2f' % q['ms_per_step'], q['ms_per_step_all'])" | tee -a $R/gpurun_out/pcie_ab.txt
done

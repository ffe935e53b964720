#!/bin/bash
# Copies a tools/round_measure.sh run (gpurun_out/m_TAG) into profiles/TAG_*
# and refreshes profiles/traffic.json from its PMC passes.
tag=$1; m=gpurun_out/m_$tag
set -e
for c in c2 c4_mfma c4_unweighted c4_valu c5 c4_rehearse; do [ -f $m/bench_$c.log ] || continue; grep '^{"metric"' $m/bench_$c.log > profiles/${tag}_bench_$c.json; done
cp $m/prof/c4_kernel_stats.csv profiles/${tag}_c4_kernel_stats.csv
cp $m/prof/c4_kernel_trace.csv profiles/${tag}_c4_kernel_trace.csv
tail -4 $m/gpu_tests.txt > profiles/${tag}_gpu_tests.txt
python tools/pmc_summary.py $m/pmc > profiles/${tag}_pmc_summary.txt
for p in fetch write l2 sq; do cp $m/pmc/$p/${p}_counter_collection.csv profiles/${tag}_pmc_$p.csv; done
mkdir -p profiles/${tag}_cli_e2e && cp $m/cli_e2e/*.log profiles/${tag}_cli_e2e/
python tools/traffic_json.py $m/pmc c4/mfma "profiles/${tag}_pmc_{fetch,write,l2}.csv (rocprofv3 --pmc, separate passes, bench.py --steps 5 --warmup 2)" > /dev/null
for c in c2 c4_mfma c4_unweighted c4_valu c5 c4_rehearse; do [ -f profiles/${tag}_bench_$c.json ] || continue
  python3 -c "import json;d=json.load(open('profiles/${tag}_bench_$c.json'));r=d['roofline'];print('$c', 'kernel %.3f ms'%r['kernel_ms'], 'step %.3f ms'%d['ms_per_step'], '%.3g pairs/s'%d['value'], 'frac %.3f'%r['frac'])"
done
cat profiles/${tag}_pmc_summary.txt

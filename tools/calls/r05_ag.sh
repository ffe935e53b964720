#!/bin/bash
# round-5 GPU call AG: host time per step of the rehearsed 1/8 shard (cProfile)
out=gpurun_out/r05ag; mkdir -p $out; export TMPDIR=/tmp
tools/gpu_step.sh 200 $out/shard8_prof.log python -m cProfile -o $out/shard8.prof bench.py --rehearse-dist --rehearse-shard 8 \
  --steps 1000 --warmup 20 --no-cpu-baseline || exit $?
python3 -c "
import pstats; p=pstats.Stats('$out/shard8.prof'); p.sort_stats('tottime').print_stats(25)" > $out/shard8_tottime.txt
python3 -c "
import pstats; p=pstats.Stats('$out/shard8.prof'); p.sort_stats('cumulative').print_stats('dist.py|api.py|distributed_c10d', 30)" > $out/shard8_cum.txt
echo done

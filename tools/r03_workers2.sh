# C2 partitions in flight, 20 timed steps each, two passes
OUT=gpurun_out/workers2; mkdir -p $OUT; export TMPDIR=/tmp
for r in a b; do for c in "1 1" "3 2" "3 3" "4 2" "4 4"; do set -- $c
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --mst-workers $1 --label-workers $2 > $OUT/c2_m$1_l$2_$r.json.log 2>&1 || { echo "m$1 l$2 failed"; exit 1; }
done; done
echo done

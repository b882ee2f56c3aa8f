# Profile evidence of one round: default SC and SCL bench lines, rocprofv3 kernel statistics and the
# FETCH_SIZE / WRITE_SIZE passes.  usage: bash tools/prof_round.sh TAG   (e.g. r01i)
# Traces go to /tmp on the box; only the *_stats.csv summaries are copied to gpurun_out/.
set -e
TAG=${1:?usage: prof_round.sh TAG}
cd /root/repo
export TMPDIR=/tmp
T=/tmp/${TAG}_prof
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_sc.json 2> gpurun_out/${TAG}_bench_sc.err
timeout -k 10 300 python bench.py --decoder scl > gpurun_out/${TAG}_bench_scl.json 2> gpurun_out/${TAG}_bench_scl.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/sc -o sc -- python3 bench.py --steps 300 --no-cpu-baseline > gpurun_out/${TAG}_prof_sc.json 2> gpurun_out/${TAG}_prof_sc.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T/scl -o scl -- python3 bench.py --decoder scl --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof_scl.json 2> gpurun_out/${TAG}_prof_scl.err
for f in $(find $T -name "*_stats.csv"); do cp "$f" gpurun_out/${TAG}_$(basename $(dirname $f))_$(basename $f); done
ls -la gpurun_out
# HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH HBM section)
for dec in sc scl; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $T/pmc_${dec}_$c -o run -- python3 bench.py --decoder $dec --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/${TAG}_pmc_${dec}_$c.err
    cp $(find $T/pmc_${dec}_$c -name "*counter_collection.csv") gpurun_out/${TAG}_pmc_${dec}_$c.csv
  done
done
ls -la gpurun_out

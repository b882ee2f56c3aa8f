# Round-5 A/B batch: SCL X2 variants, exact-f SC variants, calibration micros.  Each step under its
# own timeout; the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
SCL_ROUNDS=3 SCL_REPS=10 timeout -k 10 300 python -u tools/scl_variants.py time > $O/r05b_scl_x2_ab.txt 2>&1 || { cat $O/r05b_scl_x2_ab.txt; exit 1; }
cat $O/r05b_scl_x2_ab.txt
timeout -k 10 300 python -u tools/sc_ab.py run base old root1 --fm 1 --rounds 5 > $O/r05b_sc_exact_ab.txt 2>&1 || { cat $O/r05b_sc_exact_ab.txt; exit 1; }
cat $O/r05b_sc_exact_ab.txt
timeout -k 10 120 ./tools/micro/valu_cycles > $O/r05b_valu_cycles.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/micro/chain_latency > $O/r05b_chain_latency.txt 2>&1 || exit 1
cat $O/r05b_valu_cycles.txt $O/r05b_chain_latency.txt

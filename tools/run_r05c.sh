# Round-5 A/B batch 2: SCL X2 (level-range fix), exact-f SC root mode at two shapes, configs[1]
# lanes per codeword, calibration micros.  Each step under its own timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
SCL_ROUNDS=3 SCL_REPS=10 timeout -k 10 300 python -u tools/scl_variants.py time > $O/r05c_scl_x2_ab.txt 2>&1 || { cat $O/r05c_scl_x2_ab.txt; exit 1; }
cat $O/r05c_scl_x2_ab.txt
timeout -k 10 300 python -u tools/sc_ab.py run base root1 old --fm 1 --rounds 5 > $O/r05c_sc_exact_ab_1024.txt 2>&1 || { cat $O/r05c_sc_exact_ab_1024.txt; exit 1; }
timeout -k 10 300 python -u tools/sc_ab.py run base root1 --fm 1 --k 128 --n 256 --rounds 5 > $O/r05c_sc_exact_ab_256.txt 2>&1 || { cat $O/r05c_sc_exact_ab_256.txt; exit 1; }
timeout -k 10 300 python -u tools/sc_ab.py run base g8 g16 --k 128 --n 256 --bs 4096 --rounds 7 > $O/r05c_sc_c1_lanes_ab.txt 2>&1 || { cat $O/r05c_sc_c1_lanes_ab.txt; exit 1; }
cat $O/r05c_sc_exact_ab_1024.txt $O/r05c_sc_exact_ab_256.txt $O/r05c_sc_c1_lanes_ab.txt
timeout -k 10 120 ./tools/micro/valu_cycles > $O/r05c_valu_cycles.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/micro/chain_latency > $O/r05c_chain_latency.txt 2>&1 || { cat $O/r05c_chain_latency.txt; exit 1; }
tail -4 $O/r05c_valu_cycles.txt; cat $O/r05c_chain_latency.txt
timeout -k 10 60 ./tools/micro/x2_check > $O/r05c_x2_check.txt 2>&1; cat $O/r05c_x2_check.txt

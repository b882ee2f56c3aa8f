# Round-5 A/B: exact-f SC with a fixed llr_max range per code object (PL_EXF_RANGE) and the
# lane-level f inlined.  Each step under its own timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/sc_ab.py run base r1 r1i --fm 1 --rounds 5 > $O/r05f_sc_exact_ab_1024.txt 2>&1 || { cat $O/r05f_sc_exact_ab_1024.txt; exit 1; }
timeout -k 10 300 python -u tools/sc_ab.py run base r1 r1i --fm 1 --k 128 --n 256 --rounds 5 > $O/r05f_sc_exact_ab_256.txt 2>&1 || { cat $O/r05f_sc_exact_ab_256.txt; exit 1; }
cat $O/r05f_sc_exact_ab_1024.txt $O/r05f_sc_exact_ab_256.txt

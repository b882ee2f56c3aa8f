# Round-5 A/B: exact-f SC with f_exact / f_exact2 inlined too (PL_EXF_INLINE), fixed-range base.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/sc_ab.py run base fi --fm 1 --rounds 5 > $O/r05g_sc_exact_ab_1024.txt 2>&1 || { cat $O/r05g_sc_exact_ab_1024.txt; exit 1; }
cat $O/r05g_sc_exact_ab_1024.txt

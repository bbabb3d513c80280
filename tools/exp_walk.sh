# GPU box: queued vs plain list walk in k_pairs_half (CF_PAIRWALK): bitwise A/B, timing, tests
cd $GRAFT_REPO_ROOT
o=gpurun_out/walk; mkdir -p $o
L=openmm-chargeflux_amd/libchargeflux_hip.so
CF_PAIRWALK=0 timeout -k 10 300 python -u tools/ab_bits.py run $L $o/plain.npz > $o/ab0.log 2>&1 || { tail -20 $o/ab0.log; exit 1; }
CF_PAIRWALK=1 timeout -k 10 300 python -u tools/ab_bits.py run $L $o/queued.npz > $o/ab1.log 2>&1 || { tail -20 $o/ab1.log; exit 1; }
python -u tools/ab_bits.py cmp $o/plain.npz $o/queued.npz | tail -4
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 40 --warmup 5"
for w in 1 0 1 0; do
  CF_PAIRWALK=$w timeout -k 10 120 $B > $o/b_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$o/b_tmp.json')); k=d['kernels_ms_per_step']; print('walk=$w', d['ms_per_step'], d.get('ms_per_force_eval'), k['direct_pairs'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_parity.py tests/test_gpu_triclinic.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; exit $rc

# GPU box: bitwise A/B of abl/head (a previous commit's build) against the working tree's library
# (default settings, and with CF_OVERLAP=0: the one-stream launch order)
cd $GRAFT_REPO_ROOT
o=gpurun_out/abh; mkdir -p $o
timeout -k 10 300 python -u tools/ab_bits.py run abl/head/libchargeflux_hip.so $o/head.npz > $o/a.log 2>&1 || { tail -20 $o/a.log; exit 1; }
timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $o/new.npz > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
CF_OVERLAP=0 timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $o/new1s.npz > $o/c.log 2>&1 || { tail -20 $o/c.log; exit 1; }
echo "== head vs new (default)"; python -u tools/ab_bits.py cmp $o/head.npz $o/new.npz | grep -v identical
echo "== head vs new (CF_OVERLAP=0)"; python -u tools/ab_bits.py cmp $o/head.npz $o/new1s.npz | grep -v identical
exit 0

# GPU box: bitwise A/B of abl/head (a previous commit's build) against the working tree's library
cd $GRAFT_REPO_ROOT
o=gpurun_out/abh; mkdir -p $o
timeout -k 10 300 python -u tools/ab_bits.py run abl/head/libchargeflux_hip.so $o/head.npz > $o/a.log 2>&1 || { tail -20 $o/a.log; exit 1; }
timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $o/new.npz > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
python -u tools/ab_bits.py cmp $o/head.npz $o/new.npz | tail -8

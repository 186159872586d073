export RSE_JIT_CACHE_DIR=$PWD/jitcache
T16="python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --field 16 --k 20 --p 8 --shard-mib 4 --stripes 128"
bash tools/gpu_session.sh \
 "pmc_recon8:500:bash tools/pmc_kernel_session.sh recon8 bitslice_recon_kernel $T16 --op reconstruct --erase 0,1,2,3,4,5,6,7 --patterns 0" \
 "pmc_enc16:500:bash tools/pmc_kernel_session.sh enc16 bitslice_kernel $T16" \
 "pmc_wide50:500:bash tools/pmc_kernel_session.sh wide50 rse_jit_wide python3 tools/tune.py --rounds 1 --nt-only --shapes 0:0 --k 50 --p 20 --shard-mib 1 --stripes 64"

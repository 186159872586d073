T="python -u tools/tune.py --op reconstruct --rounds 3 --nt-only --bitslice 1 --patterns 1,0 --shapes 4096:1,8192:1 --k 10 --p 4 --erase 0,1"
bash tools/gpu_session.sh \
 "rec64:300:$T --stripes 64" \
 "rec448:300:$T --stripes 448" \
 "enc448:300:python -u tools/tune.py --k 10 --p 4 --stripes 448 --rounds 3 --shapes 4096:1 --nt-only" \
 "host_e2e:400:python -u tools/host_e2e.py --stripes 8 --reps 3"

/* rse_hip_tune.h -- tuning and A/B switches of librse_hip.so (not part of the
 * drop-in surface: include/rse_hip.h has the options a caller needs).
 *
 * rse_set_option refuses these keys with RSE_ERR_INVALID_ARGUMENT unless the
 * process environment has RSE_TUNE=1 (tests/conftest.py and the tools/ that
 * A/B them set it); rse_get_option reads them always.  Each selects among
 * kernels or launch shapes that give the same bytes; the defaults are the
 * measured best.  Options that shape run-time modules apply to
 * modules built after they are set.  The timing splits that write wrong bytes
 * (RSE_OPT_RECON_PAIRS 4 / 5, key 47) exist only in the -DRSE_TUNE_SPLITS
 * build (make tune). */
#ifndef RSE_HIP_TUNE_H
#define RSE_HIP_TUNE_H

#define RSE_OPT_NONTEMPORAL 1       /* 1: streaming (nt) loads/stores of shard bytes */
#define RSE_OPT_GRID_X 2            /* table kernels: workgroups per stripe row; bit-sliced
                                       kernels: total workgroups; 0 = automatic */
#define RSE_OPT_STRIPES_IN_FLIGHT 3 /* stripes coded concurrently (grid.y); 0 = all */
#define RSE_OPT_KERNEL_VARIANT 4    /* compiled variant of a tuned shape; -1 = tuned default */
#define RSE_OPT_BITSLICE 5          /* 1: bit-sliced kernels for compiled codecs (default) */
#define RSE_OPT_JIT_CSE 13          /* GF(2^16) specialised XOR networks: up to this many shared
                                       subexpressions per input (0..32, default 32), for modules
                                       built after */
#define RSE_OPT_WIDE_LDS 14         /* wide-codec modules built after: 1 (default) each wave slices
                                       1/W of the inputs and shares the planes through LDS; 0 every
                                       wave slices every input */
#define RSE_OPT_RECON_MIX 17        /* syndrome reconstruct of the compiled-in codecs, the e x e
                                       mixing: 3 (default) bit-sliced Horner's rule, four steps per
                                       mask word unrolled; 2 the same one step at a time, 1 bit-sliced
                                       doubling chains above 4 rows, 0 v_perm tables (A/B) */
#define RSE_OPT_WIDE_SPLIT 18       /* outputs per wave of the one-module kernels (2..8; 0, the
                                       default: 8, and 4 for GF(2^8) codecs past 48 parity rows):
                                       a codec with more parity rows than this (but <= 8 x this)
                                       is coded by W waves sharing each input chunk */
#define RSE_OPT_WIDE_BALANCE 19     /* 1 (default): W at least 4 (p >= 4) and a power of two, so a
                                       CU's 4 SIMDs hold equally many waves of the wide kernels;
                                       0: W = ceil(p / split) */
#define RSE_OPT_WIDE_OCCUPANCY 20   /* minimum waves per SIMD the wide kernels are compiled for:
                                       0 (default) = 2, or 2..4 */
#define RSE_OPT_HOST_COPY_2D 21     /* host pipeline (*_host_flat): 1 (default) one 2D copy per run of
                                       equally spaced shards of the caller buffer, 0 one copy per shard */
#define RSE_OPT_JIT_EXACT 23        /* run-time networks built after: 1 (default) temporaries chosen by
                                       exact fewest-source decompositions (rse_netgen.hpp factor8 /
                                       factor16), 0 the pair/triple greedy (A/B) */
#define RSE_OPT_WIDE_DEPTH 26        /* wide-codec modules built after: 4 KiB inputs each wave keeps in
                                       flight (1..4, default 1; past a chunk's last round, the next
                                       chunk's first ones) */
#define RSE_OPT_RECON_DEPTH 27       /* syndrome reconstruct: inputs in flight per lane (1..4) */
#define RSE_OPT_RECON_PAIRS 28       /* syndrome reconstruct at 8 sigma rows on wave pairs (4 rows
                                        each, planes shared through LDS, 3 waves per SIMD): 8
                                        (default) by field -- GF(2^8) as 2, GF(2^16) as 1; 1 one
                                        pair per workgroup with two inputs in flight per wave, 2
                                        two pairs per workgroup
                                        (compiled codecs; run-time ones use two); 0: one wave holds
                                        all 8 rows; A/B variants of the compiled codecs (one pair):
                                        3 next unit prefetched, 6 compact mixing, 7 one input in
                                        flight per wave (round 3's kernel).  4 / 5 (timing
                                        splits that skip the Horner steps / data networks, which
                                        write wrong bytes) exist only in tools/tune.py's
                                        -DRSE_TUNE_SPLITS build: this library refuses them with
                                        RSE_ERR_INVALID_ARGUMENT and keeps its setting */
#define RSE_OPT_WIDE_PAIRS 29        /* wide GF(2^8) modules built after: 1 (default) XOR networks
                                        over pairs of inputs (temporaries may combine both), coded two
                                        inputs at a time; 0: one input at a time */
#define RSE_OPT_SYNC_EVENT 30        /* 1: verify calls wait on an event recorded after their
                                        kernels instead of synchronising the stream (A/B; 0 default) */
#define RSE_OPT_SPIN_WAIT 31         /* 1 (default): a verify that is one check-kernel launch
                                        (compiled or run-time specialised codecs) signals its
                                        completion through a word of pinned host memory, which the
                                        call polls instead of synchronising the stream; 0:
                                        synchronise (A/B) */
#define RSE_OPT_HOST_DIRECT 32       /* 1 (default): a *_host call on one stripe that moves at most
                                        2 MiB goes through one pinned staging buffer (CPU copies,
                                        one DMA each way) instead of the chunk pipeline's per-shard
                                        copies; 0: always the pipeline (A/B) */
#define RSE_OPT_SUB_CHUNKS 33        /* 1 (default): shards of exactly 1 or 2 KiB run on the
                                        bit-sliced kernels, a 4 KiB chunk taking 4 or 2 stripes'
                                        shards; 0: the table kernels (A/B) */
#define RSE_OPT_SUBFIELD 34          /* 1 (default): a GF(2^16) codec (read at rse_codec_new) or
                                        coding pass whose coefficients all lie in the GF(2^8)
                                        subfield -- every codec of at most 256 shards -- codes
                                        each byte in GF(2^8): the same bytes, half the work;
                                        0: GF(2^16) kernels (A/B) */
#define RSE_OPT_RECON_W4_MIN 37      /* a pattern's first use on shards with 4 KiB chunks past their
                                        16 KiB ones (or shorter than 16 KiB): the syndrome kernels
                                        code those chunks when k x outputs >= this (default 64;
                                        GF(2^16) proper always), else the table kernels do */
#define RSE_OPT_WIDE_HALF 38         /* wide GF(2^8) modules with paired networks built after: 1
                                        (default) each wave codes 2 KiB chunks, one 8-plane group
                                        per lane (half the accumulators: 8 outputs per wave fit in
                                        registers); 0: 4 KiB chunks, two groups per lane */
#define RSE_OPT_WIDE_GRID 44          /* wide-module launches: -1 fixed workgroup counts (8192
                                        GF(2^8), 16384 GF(2^16)); m > 0: m x the workgroups the
                                        device holds at once (occupancy of the module); 0
                                        (default): 1 x that for 1 / 2 KiB shards of codecs with
                                        k x p >= 1000, fixed counts otherwise */
#define RSE_OPT_WIDE_BLOCK_INPUTS 46  /* codecs past one wide module (k + 2p > 480: GF(2^16) past
                                        256 shards): a chain of wide modules over blocks of at
                                        most this many data inputs, each coding every output
                                        (default 128); 0: modules of 8 outputs x 32 inputs */
#define RSE_OPT_DISPATCH_LANE_UNITS 49 /* dispatcher: a request takes ceil(units / (this x 512))
                                        of the resident workgroups, units = 16-byte vectors x
                                        outputs (default 1); one workgroup up to 1024 units */
#define RSE_OPT_SUB_DEPTH 50          /* run-time modules built after: inputs in flight per wave of
                                        their 1 / 2 KiB-shard kernels (1: bitslice_body; 2..4,
                                        default 4: rse_sub_ext.hpp) */
#define RSE_OPT_FFT 51                /* 1 (default): GF(2^8) codecs with k = p = 16, 32 or 64
                                        (benches/bandwidth.rs's 16+16 .. 64+64) encode, verify and
                                        rebuild all data shards from the parity shards on additive-FFT
                                        kernels ((k/2) log2 k butterflies per transform instead of
                                        k x p coefficient networks; same bytes); 0: the wide modules */
#define RSE_OPT_HOST_QUEUES 52        /* host pipeline (*_host_flat) streams: 1 (default) the D2H
                                         stream at high priority, on hardware queues no default-
                                         priority stream shares, so the D2H copies never hold up
                                         the H2D copies whatever other streams the process holds;
                                         0 plain streams (A/B) */
#define RSE_OPT_HOST_ZC_OUT 53        /* host pipeline (*_host_flat, reconstruct_host*): 1 (default)
                                         the shards an encode or reconstruct writes, when they are
                                         pinned device-mapped host memory, are stored in place by
                                         the kernel (no D2H copies); 0 D2H copies from the ring */

#endif /* RSE_HIP_TUNE_H */

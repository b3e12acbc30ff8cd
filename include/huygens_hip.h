/*
 * huygens_hip.h -- C ABI of libhuygens_hip.so, the MI355X (gfx950) bank engine.
 *
 * This is the drop-in boundary for the per-sample bank hot path of
 * amcerbu/huygens (namespace soundmath, header-only C++17).  The reference has
 * no .so and no plugin registry: its "operator API" is operator() + tick() +
 * setters on class templates.  Each entry point below names the reference
 * member it replaces (file:line under /root/reference).  The C++ wrappers in
 * include/soundmath/ *.h restore the reference class names and signatures on
 * top of this ABI.
 *
 * Conventions
 *   - Opaque handles; every call returns int: HZ_OK (0) or a negative HZ_E_*.
 *     The reference aborts through Eigen asserts on out-of-range indices
 *     (tests/build.sh:8 builds without NDEBUG); this ABI never aborts and
 *     reports HZ_E_RANGE instead.  hz_last_error() gives a per-thread message.
 *   - Setters are staged on the host and applied at the next process call
 *     boundary (block-granular; the reference mutates state from the MIDI
 *     thread with no synchronisation, tests/filterbank.cpp:236-244).
 *   - *_process() take HOST pointers and are synchronous (H2D, kernels, D2H).
 *     *_process_device() take DEVICE pointers and are asynchronous on the
 *     handle's HIP stream (hz_*_set_stream / hz_*_get_stream).
 *   - No torch types; plain pointers and sizes only.
 */
#ifndef HUYGENS_HIP_H
#define HUYGENS_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HZ_OK 0
#define HZ_E_INVALID (-1) /* bad argument (null handle, n < 0, bad order ...) */
#define HZ_E_RANGE (-2)   /* index out of range (reference: Eigen assert abort) */
#define HZ_E_HIP (-3)     /* a HIP runtime call failed                        */
#define HZ_E_NODEV (-4)   /* no gfx950 device visible                         */
#define HZ_E_ALLOC (-5)   /* device or host allocation failed                 */
#define HZ_E_UNSUPPORTED (-6)
#define HZ_E_STATE (-7)   /* the call needs state the handle does not keep        */

/* per-band distortion functors replacing T(*)(T) in
 * Filterbank::operator()(T, T(*)(T)) (src/filterbank.h:133-139) */
#define HZ_DIST_NONE 0
#define HZ_DIST_SOFTCLIP 1 /* tests/filterbank.cpp:158-166, param = width      */
#define HZ_DIST_SATURATE 2 /* tests/filterbank.cpp:173-176                     */
#define HZ_DIST_LIMITER 3  /* src/wave.h:150 limiter, FUNCTIONAL: 2/PI atan(x) */
/* The reference's demos pass &softclip, which resolves to the one-argument overload
 * softclip(sample) = softclip(sample, 0.125) (tests/filterbank.cpp:168-171): the width a drop-in
 * F(x, HZ_DIST_SOFTCLIP) uses when none is given. */
#define HZ_SOFTCLIP_WIDTH 0.125
#define HZ_DIST_DEFAULT_PARAM(dist_id) ((dist_id) == HZ_DIST_SOFTCLIP ? HZ_SOFTCLIP_WIDTH : 0.0)

/* ---- library ---------------------------------------------------------- */
const char* hz_last_error(void);
int hz_version(void);
/* number of visible gfx950 devices (0 when none; never errors) */
int hz_device_count(void);

/* ---- Filterbank<double>  (src/filterbank.h:16-188) --------------------- */
typedef struct hz_fb hz_fb;

/* Filterbank(int order, int N, double k_p, double k_g)  filterbank.h:36-70.
 * order in [0, 4]. */
int hz_fb_create(int order, int N, double k_p, double k_g, int device, hz_fb** out);
/* band shard [band_begin, band_begin + band_count) of an N_total-band bank,
 * for one process per GPU (partial mixes are summed by the caller over RCCL);
 * setters take GLOBAL band indices and ignore bands outside the shard. */
int hz_fb_create_shard(int order, int N_total, int band_begin, int band_count, double k_p,
                       double k_g, int device, hz_fb** out);
int hz_fb_destroy(hz_fb* h);                                        /* ~Filterbank 23-33 */
/* coefficients(int n, const vector<T>& fwd, const vector<T>& back)  73-82 */
int hz_fb_coefficients(hz_fb* h, int n, const double* fwd, int nf, const double* back, int nb);
int hz_fb_boost(hz_fb* h, int n, double v);                         /* boost(int,T)   85-88 */
int hz_fb_boost_all(hz_fb* h, const double* v, int count);          /* boost(vector)  91-96 */
int hz_fb_mix(hz_fb* h, int n, double v);                           /* mix(int,T)     99-102 */
int hz_fb_mix_all(hz_fb* h, const double* v, int count);            /* mix(vector)   105-110 */
int hz_fb_open(hz_fb* h);                                           /* open()        112-116 */
/* selects the T(*)(T) of operator()(T, T(*)(T)) for subsequent process calls */
int hz_fb_set_distortion(hz_fb* h, int dist_id, double param);
/* n x { out[i] = operator()(in[i]); tick(); }  (filterbank.h:125-148) */
int hz_fb_process(hz_fb* h, const double* in, double* out, size_t n);
int hz_fb_process_device(hz_fb* h, const double* d_in, double* d_out, size_t n);
/* tick() WITHOUT a preceding operator()  (filterbank.h:142-148): origin moves and nothing is
 * computed, so the smoothers stand still and the next sample reads, as its newest history
 * row (x and every band's y), the ring row left from O+1 samples earlier (the reference's
 * rings hold O+1 rows).  The handle keeps that row after a 1-sample process call, after
 * another hz_fb_tick and at creation; after a call of n >= 2 samples or hz_fb_set_state it
 * is not kept and hz_fb_tick returns HZ_E_STATE.  (A tick() that follows operator() is
 * already part of every process call.) */
int hz_fb_tick(hz_fb* h);
/* Per-sample operator API on the GPU (hz_fb_rt.hip): T operator()(T x) / operator()(T x, dist)
 * (filterbank.h:125-139) and tick() (142-148) with the reference's exact semantics -- a repeated
 * operator() before tick() returns the cached row re-mixed (no compute); ticks without operator()
 * rotate the ring (the row O+1 samples back becomes the newest history row).  Served by the
 * device's per-sample server (hz_rt_info: one resident kernel for every handle, pinned-host
 * mailbox, a few microseconds per sample) over the handle's state in device memory; the state is
 * converted back on the next block call, state read/write or destroy.  Setters between samples
 * reach the next request as a payload (no restart).  hz_fb_sample_tick only records the tick
 * (no GPU work).  Block calls after an operator() without tick() output the cached sample first,
 * as the reference's loop does.  HZ_E_STATE for a bare tick whose ring row is unknown (see
 * hz_fb_tick). */
int hz_fb_sample(hz_fb* h, double x, int dist_id, double param, double* y);
int hz_fb_sample_tick(hz_fb* h);
/* One sample of several Filterbanks in ONE per-sample server request -- the per-channel banks of
 * tests/filterbanks.cpp:191-211 (CHANELS FFilterbank<double,864,2> ticked per sample, &softclip):
 * y[i] = operator()(x[i], dist) of handles[i] for every i, each with its own pending tick()s, as
 * count separate hz_fb_sample calls would give (the mixdown summed in another fixed order: equal to
 * rounding).  The handles share a device and an order, each appears once; count <= 12 and
 * 6 + count (order + 2) <= 62.  Setters on a member since its last sample, and switching a handle
 * between this call and hz_fb_sample, relaunch the server (tens of microseconds once). */
int hz_fb_sample_many(hz_fb* const* handles, int count, const double* x, int dist_id, double param, double* y);
/* the number of per-sample calls served when the last setter (coefficients / boost / mix / open)
 * ran: the setter applies from that call on (setters may come from another thread while samples
 * run -- every entry point holds the handle's lock; the reference's MIDI thread,
 * tests/filterbank.cpp:217-252) */
int hz_fb_setter_seq(hz_fb* h, long long* seq);
/* whether the handle is in per-sample mode, samples served, server workgroups taking part */
int hz_fb_sample_info(hz_fb* h, int* active, long long* served, int* groups);
int hz_fb_set_stream(hz_fb* h, void* hip_stream);
int hz_fb_get_stream(hz_fb* h, void** hip_stream);
int hz_fb_synchronize(hz_fb* h);
/* state = [x history (order)] [y history (N*order)] [pre,gain (N*2)] */
int hz_fb_state_size(hz_fb* h, size_t* count);
int hz_fb_get_state(hz_fb* h, double* buf, size_t count);
int hz_fb_set_state(hz_fb* h, const double* buf, size_t count);
int hz_fb_info(hz_fb* h, int* order, int* N_local, int* band_begin, int* N_total);
/* kernel geometry: waves per workgroup (4, 8, 16), bands per wave (1); 0 = default */
int hz_fb_tune(hz_fb* h, int waves_per_group, int bands_per_wave);
/* HIP-event timing of the launches of subsequent process calls, on the handle's
 * stream: total ms of the time-segment pre-pass (segment end states + carry;
 * 0 when the bank fills the GPU with bands alone), of the IIR/mixdown kernel,
 * of the cross-group reduce kernel, and the number of process launches.
 * enable > 1 (at most 64): the stationary engine's modal-path kernels run `enable`
 * times back to back between their events and the times read are per launch. */
int hz_fb_profile(hz_fb* h, int enable);
int hz_fb_profile_read(hz_fb* h, double* segment_ms, double* mix_ms, double* reduce_ms, long* launches);
/* workgroups wanted per launch before time segmentation kicks in (default: CU count) */
int hz_fb_set_target_groups(hz_fb* h, int groups);
/* Execution path of process calls.  HZ_FB_PATH_AUTO: the converged ("LTI") engine
 * whenever every band's pre-amp and gain smoother has converged to its target
 * (|pre - pin| <= 2^-60 max|pin|, same for gains) and no distortion functor is set,
 * the general engine otherwise (hz_fb_lti.h).  HZ_FB_PATH_GENERAL: always the
 * general engine.  hz_fb_last_path reports the path the last process call took
 * (HZ_FB_PATH_LTI if any of its samples went through the LTI engine). */
#define HZ_FB_PATH_AUTO 0
#define HZ_FB_PATH_GENERAL 1
#define HZ_FB_PATH_LTI 2
#define HZ_FB_PATH_RESPONSE 3
#define HZ_FB_PATH_STREAM 4
int hz_fb_set_path(hz_fb* h, int path);
int hz_fb_last_path(hz_fb* h, int* path);
/* Stationary engine (HZ_FB_PATH_RESPONSE, hz_fb_resp.hip).  Once the bank has run converged
 * (as for the LTI engine) with unchanged coefficients and targets for K samples -- K = its
 * horizon, the first multiple of 8192 with ||M^K||_inf < 2^-53 for every band's state transition
 * M (src/filterbank.h:178-179) -- the mixdown of a long call (>= 16384 samples) is one linear
 * filter of the input, out = h * x with h = sum_n gin_n (band n's impulse response at pre = pin_n),
 * truncated at K, and runs as a partitioned FFT convolution.  The band states at the call end are
 * the zero-start response of the last K inputs: computed after every call (HZ_FB_RESP_EAGER,
 * default) or when a later call / get_state / tick needs them (HZ_FB_RESP_LAZY).
 * HZ_FB_RESP_OFF keeps the per-band engines.  Env HZ_FB_RESP=0/1/2 sets the default. */
#define HZ_FB_RESP_OFF 0
#define HZ_FB_RESP_EAGER 1
#define HZ_FB_RESP_LAZY 2
int hz_fb_set_response(hz_fb* h, int mode);
/* (tuning) shortest call that runs stationary and keeps the history (0: 16384); the engine is
 * chosen when N n >= bands_per_sample (K + n) (0: 256, env HZ_FB_RESP_BANDS) */
int hz_fb_tune_response(hz_fb* h, long min_call, long bands_per_sample);
/* (tuning / A-B) the long-call convolution's structure: 0 (default) = the three-kernel path
 * (forward transforms, partition MACs, inverse transforms + band-state pass); 1 = column-split, two
 * kernels per call (hz_fb_col.h: forward transforms, partition MACs and inverse columns in one
 * kernel that keeps the window spectra on chip, then the output combine with the band-state pass)
 * for banks whose horizon is 8, 16 or 24 partitions of 2048 -- measured slower on MI355X (C2: 0.048
 * against 0.0405 ms per step).  Results agree to rounding. */
int hz_fb_tune_response_engine(hz_fb* h, int column_split);
/* the setting above, and the last stationary call's path: 1 column-split, 2 three-kernel with
 * modal band states (hz_fb_tune_modal), 0 three-kernel with the matrix-core state pass */
int hz_fb_response_engine(hz_fb* h, int* column_split_on, int* last_call_column_split);
/* Modal band states (default on): a stationary call's band states for banks whose poles sit on one
 * circle at angles on the 2 pi / 8192 grid (e.g. the resonator recipe f_i = 0.5 (i + 1) SR / N,
 * N <= 4096, one R; tests/resynthesis.cpp:48-54) come from a fold of the call's last K inputs and
 * one 8192-point DFT instead of the N O K multiply-adds of the matrix-core pass; up to 8 bands with
 * (nearly) coincident poles take direct sums.  Results agree with the matrix-core pass to rounding
 * (DESIGN.md 3.6).  on = 0: always the matrix-core pass. */
int hz_fb_tune_modal(hz_fb* h, int on);
/* the setting, whether the current bank qualifies (its states computed by the modal pass), its
 * exceptional (direct-sum) bands (-1: does not qualify) and whether the last stationary call used it */
int hz_fb_modal_info(hz_fb* h, int* on, int* qualifies, int* exceptional, int* last_call);
/* horizon K (-1: none within 2^21 samples, -2: not computed), stationary samples so far,
 * whether the band states are implicit (LAZY), stationary calls made */
int hz_fb_response_info(hz_fb* h, long* horizon, long* run, int* implicit_state, long* calls);
/* the bank response h[0 .. count) (zero past the horizon); HZ_E_UNSUPPORTED without a horizon */
int hz_fb_get_response(hz_fb* h, double* out, long count);
/* Time-range shards of the stationary engine (multi-GPU, one process per GPU): each rank owns a
 * band shard (hz_fb_create_shard) for the band states, sets the WHOLE bank's response -- the sum
 * over ranks of hz_fb_get_response(K values), K = the largest horizon of the ranks (a multiple of
 * 8192; a longer horizon than the shard's own restarts its history), e.g. one RCCL all-reduce -- with
 * hz_fb_set_bank_response, and its rank / world with hz_fb_set_time_shard.  Its stationary calls
 * then convolve only rank's run of whole 2048-sample output blocks with that response and write
 * zeros elsewhere, so the ranks' outputs still sum to the call's mix (or are gathered by range:
 * hz_fb_time_shard_info).  Every setter (also for bands of other shards) clears the bank
 * response; count 0 clears it explicitly.  Without it a call outputs all samples of its own bands. */
int hz_fb_set_bank_response(hz_fb* h, const double* resp, long count);
int hz_fb_set_time_shard(hz_fb* h, int rank, int world);
/* zero_outside = 1 (default): a time-sharded stationary call writes zeros outside its share, so the
 * ranks' outputs sum (one reduce) to the call's mix; 0: it leaves the rest of the output untouched --
 * the shares are disjoint and final, nothing to reduce (bench.py N > 1: no data-path collective;
 * huygens_amd.shard.ShareGather collects them on one rank with 1/world of the output per rank). */
int hz_fb_set_time_shard_fill(hz_fb* h, int zero_outside);
/* The engine choice of time-sharded handles is collective: such a handle runs its per-band
 * engines (band-shard partial mixes) until the caller arms it, and runs stationary exactly when
 * armed -- an armed handle whose call cannot be stationary returns HZ_E_STATE instead of
 * diverging from its peers.  Protocol (huygens_amd/shard.py arm_when_ready): after a call, every
 * rank asks hz_fb_stationary_ready(n) (would a call of n samples be stationary on this handle),
 * all-reduces the flag with MIN and passes the result to hz_fb_arm_time_shard.  Setters,
 * hz_fb_set_bank_response and hz_fb_set_time_shard disarm. */
int hz_fb_stationary_ready(hz_fb* h, long n, int* ready);
int hz_fb_arm_time_shard(hz_fb* h, int armed);
/* for a stationary call of n samples: whether it is time-sharded, and its output range */
int hz_fb_time_shard_info(hz_fb* h, int* active, long* first, long* count, long n);
/* Streaming calls (HZ_FB_PATH_STREAM, hz_fb_stream.hip) -- the reference's 1024-sample audio
 * callback (tests/resynthesis.cpp:33-42 over src/filterbank.h:125-148).  A call of exactly 1024
 * samples on a stationary bank (as above: converged, unchanged for K samples, K <= 2^17, no
 * distortion, no time shard) runs as ONE kernel launch: a partitioned overlap-save convolution
 * with 1024-sample partitions whose window spectra stay on the device between calls.  1024-sample
 * calls on the per-band engines keep the history for it; band states stay implicit after a
 * streamed call (in every response mode) until a later call, get_state, tick or a setter needs
 * them.  hz_fb_tune_stream(h, 0) keeps such calls on the per-band engines (default 1). */
int hz_fb_tune_stream(hz_fb* h, int enable);
/* engine enabled, its call length (1024), streamed calls made, history currently in its ring */
int hz_fb_stream_info(hz_fb* h, int* enabled, long* block, long* calls, int* history_in_ring);
/* LTI engine geometry: (chunk length, bands per wave, waves per group) in
 * {(16,1,16), (32,1,16), (64,1,16), (128,1,16)}; 0s = by call length (default: 128 for calls
 * of >= 4 x 8192 samples on banks that fill the chip with <= 2 time segments, 64 from
 * 2 x 4096 samples, 32 from 2 x 2048, else 16) */
int hz_fb_tune_lti(hz_fb* h, int chunk, int bands_per_wave, int waves_per_group);
/* (diagnostics) plan of the last LTI launch: time segments, segment-prepass tiles skipped
 * at the head of each segment (the horizon prepass; 0 = full prepass), fine prepass parts */
int hz_fb_lti_plan(hz_fb* h, long* nseg, long* skip_tiles, int* fine_parts);
/* (diagnostics) chunk length L of the last LTI launch (16, 32, 64 or 128; 0 before any) */
int hz_fb_lti_last_chunk(hz_fb* h, int* chunk);

/* ---- the per-sample server (hz_rt.hip) ----------------------------------------
 * One resident kernel per device serves the per-sample calls of Filterbank (hz_fb_sample),
 * Delay / Delaybank (hz_dly_sample) and Granulator (hz_gran_sample) through a pinned-host
 * mailbox, on a stream of the highest priority; it leaves after 2 ms without a request and is
 * relaunched on demand.  Statistics: requests served, launches, currently resident. */
int hz_rt_info(int device, long long* requests, long long* launches, int* active);

/* ---- Oscbank<double,N>  (src/oscbank.h:15-97, src/multichannel.h:16-159) -- */
typedef struct hz_osc hz_osc;

/* Oscbank(double k = 2.0/SR)  oscbank.h:37-47 (k's stiffness is unused there too) */
int hz_osc_create(int N, double k, int device, hz_osc** out);
/* oscillators [begin, begin+count) of an N_total bank; indices stay global */
int hz_osc_create_shard(int N_total, int begin, int count, double k, int device, hz_osc** out);
int hz_osc_destroy(hz_osc* h);                                   /* ~Oscbank 30-34 */
/* freqmod(int index, T hz)  49-56: out-of-range indices are ignored (HZ_OK) */
int hz_osc_freqmod(hz_osc* h, int index, double hz);
int hz_osc_activate(hz_osc* h, const int* idx, int count);      /* multichannel.h:87-92 */
int hz_osc_deactivate(hz_osc* h, const int* idx, int count);    /* multichannel.h:95-100 */
int hz_osc_open(hz_osc* h);                                      /* multichannel.h:103-109 */
int hz_osc_close(hz_osc* h);                                     /* multichannel.h:112-118 */
int hz_osc_active_count(hz_osc* h, int* count);
/* n x { mix[t] = mixdown(); per_band[t][:] = operator()(); tick(); }  (65-90, 59-63)
 * mix: 2n doubles (complex interleaved) or NULL; per_band: 2nN doubles or NULL */
int hz_osc_fill(hz_osc* h, double* mix, double* per_band, size_t n);
int hz_osc_fill_device(hz_osc* h, double* d_mix, double* d_per_band, size_t n);
/* operator()(): the N phasors (2N doubles, complex interleaved) */
int hz_osc_phases(hz_osc* h, double* z);
/* mixdown() of the current phasors (sum over the active set in index order) without a tick */
int hz_osc_mixdown(hz_osc* h, double* mix);
int hz_osc_set_phases(hz_osc* h, const double* z);
int hz_osc_set_stream(hz_osc* h, void* hip_stream);
int hz_osc_synchronize(hz_osc* h);
int hz_osc_set_target_groups(hz_osc* h, int groups);
int hz_osc_profile(hz_osc* h, int enable);
int hz_osc_profile_read(hz_osc* h, double* ms, long* launches);

/* ---- Additive<double>  (src/additive.h:11-71 + Minimizer note API,
 *      src/minimizer.h:111-187; physics() is out of scope) ------------------- */
typedef struct hz_add hz_add;
/* Additive(Wave* = &cycle, voices, overtones, decay, harmonicity = 1, k = 0.1)  additive.h:24-36 */
int hz_add_create(int voices, int overtones, double decay, double harmonicity, double k, int device,
                  hz_add** out);
/* overtones [o_begin, o_begin + o_count) of every voice (one process per GPU; the
 * note API is replicated on every rank so voice allocation agrees) */
int hz_add_create_shard(int voices, int overtones, int o_begin, int o_count, double decay, double harmonicity,
                        double k, int device, hz_add** out);
int hz_add_destroy(hz_add* h);
int hz_add_request(hz_add* h, double fundamental, double amplitude, int* voice);   /* minimizer.h:111-158 */
int hz_add_release(hz_add* h, int voice);                                          /* 161-172, -1 = all */
int hz_add_makenote(hz_add* h, double pitch, double amplitude, int* voice);        /* 174-179 */
int hz_add_endnote(hz_add* h, double pitch);                                       /* 182-187 */
/* n x { out[t] = operator()(); tick(); }  additive.h:38-62 (tests/additive.cpp:27-37).
 * Per-sample calls (n < 64: the drop-in's operator() / tick()) are served from a speculative
 * block: the next 1024 samples rendered at once from a snapshot of the state (the output needs no
 * input); a setter, a longer fill or a device fill first rolls the engine back to the consumed
 * sample (snapshot restored, that many samples re-rendered), so the samples are exactly those of
 * the per-sample sequence.  The same holds for Sinusoids (hz_sin_fill), Bowl (hz_bowl_render /
 * hz_bowl_fill) and Oscbank (hz_osc_fill with n = 1, hz_osc_phases, hz_osc_mixdown). */
int hz_add_fill(hz_add* h, double* out, size_t n);
/* speculative blocks rendered, rollbacks (a setter inside a block), block length */
int hz_add_lookahead_info(hz_add* h, long* blocks, long* rollbacks, long* block_len);
int hz_add_fill_device(hz_add* h, double* d_out, size_t n);
int hz_add_set_stream(hz_add* h, void* hip_stream);
int hz_add_set_target_groups(hz_add* h, int groups);
int hz_add_profile(hz_add* h, int enable);
int hz_add_profile_read(hz_add* h, double* ms, long* launches);

/* ---- Sinusoids<double>  (src/sinusoids.h:10-79), waveform cycle ------------ */
typedef struct hz_sin hz_sin;
/* Sinusoids(Wave*, fundamental, overtones, decay, harmonicity = 1, k = 2.0/SR) 16-31 */
int hz_sin_create(double fundamental, int overtones, double decay, double harmonicity, double k, int device,
                  hz_sin** out);
int hz_sin_destroy(hz_sin* h);
int hz_sin_fundmod(hz_sin* h, double target);    /* 67-68 */
int hz_sin_decaymod(hz_sin* h, double target);   /* 61-62 */
int hz_sin_harmmod(hz_sin* h, double target);    /* 64-65 */
/* n x { out[t] = operator()(); tick(); }  34-57 */
int hz_sin_fill(hz_sin* h, double* out, size_t n);
int hz_sin_fill_device(hz_sin* h, double* d_out, size_t n);

/* ---- Bowl<T>  (src/bowl.h:10-74), T = double (is_float 0) or float (1) ----
 * Bowl(int overtones, const vector<T>& f, const vector<T>& a, const vector<T>& d,
 *      Wave<T>* form = &cycle)  bowl.h:16-23; the form is cycle (sin 2 PI p) for double and
 * the Wave<float> lambda sin(2 PI p) for float (&cycle does not compile for float). */
typedef struct hz_bowl hz_bowl;
int hz_bowl_create(int overtones, const double* f, const double* a, const double* d, int count, int is_float,
                   int device, hz_bowl** out);
int hz_bowl_destroy(hz_bowl* h);
int hz_bowl_trigger(hz_bowl* h);                                        /* 25-28 */
int hz_bowl_fill(hz_bowl* h, float* buffer, size_t bsize);              /* int fill(float*, int) 50-63 */
int hz_bowl_fill_device(hz_bowl* h, float* d_buffer, size_t bsize);
/* n x { out[j] = operator()(); tick(); }  30-48 (T's precision, widened to double) */
int hz_bowl_render(hz_bowl* h, double* out, size_t n);
int hz_bowl_render_device(hz_bowl* h, double* d_out, size_t n);
int hz_bowl_phase(hz_bowl* h, double* phase);
int hz_bowl_set_stream(hz_bowl* h, void* hip_stream);
int hz_bowl_set_target_groups(hz_bowl* h, int groups);
int hz_bowl_profile(hz_bowl* h, int enable);
int hz_bowl_profile_read(hz_bowl* h, double* ms, long* launches);

/* ---- Delay<T> / Delaybank<T,N>  (src/delay.h:10-108 over src/buffer.h:9-86) ----
 * A Delaybank is N independent Delay<T> lines (the reference's src/delaybank.h:15-54 is a
 * non-functional stub); Delay<T> is the N = 1 case.  T = double (is_float 0)
 * or float (1).  Delaybank(uint sparsity, uint time): rings of time+1 samples per line
 * (delay.h:21-35); time < 2^31 - 1.  Taps are (uint time, T gain) pairs; a zero-time
 * feedback tap becomes {0,0} (delay.h:48-51, 64-67).  Ring indexing is bit-exact with
 * buffer.h:40-47, including the uint32 wrap of delays longer than the ring. */
typedef struct hz_dly hz_dly;
int hz_dly_create(int lines, unsigned sparsity, unsigned time, int is_float, int device, hz_dly** out);
int hz_dly_destroy(hz_dly* h);
/* coefficients(forward, back) of one line (delay.h:37-56); missing taps are zeroed */
int hz_dly_coefficients(hz_dly* h, int line, const unsigned* fwd_time, const double* fwd_gain, int nf,
                        const unsigned* back_time, const double* back_gain, int nb);
int hz_dly_modulate_forward(hz_dly* h, int line, unsigned n, unsigned time, double gain); /* 59-60 */
int hz_dly_modulate_back(hz_dly* h, int line, unsigned n, unsigned time, double gain);    /* 63-68 */
/* n x { y_k = line_k(x); tick(); } for every line (delay.h:71-97).  Samples are T.
 * in: mono [n] (in_per_line 0) or line-major [N][n]; out: line-major [N][n] (mix 0) or
 * the mixdown sum_k y_k / N, summed in line order in T (mix 1). */
int hz_dly_process(hz_dly* h, const void* in, void* out, size_t n, int in_per_line, int mix);
int hz_dly_process_device(hz_dly* h, const void* d_in, void* d_out, size_t n, int in_per_line, int mix);
/* one sample of every line, `y_k = line_k(x); tick();` (delay.h:71-97), through the device's
 * per-sample server (a resident kernel shared by every handle of the process; no launch per
 * sample): in = one T (in_per_line 0) or N T, out = N T.  Bit-identical to hz_dly_process(n = 1). */
int hz_dly_sample(hz_dly* h, const void* in, void* out, int in_per_line);
/* tick() without operator() (delay.h:92-97), `count` times: both rings' origins move and no
 * slot is written (the stale samples stay, as in the reference) */
int hz_dly_tick(hz_dly* h, unsigned long count);
int hz_dly_origin(hz_dly* h, unsigned* origin);            /* Buffer::origin after the last call */
int hz_dly_info(hz_dly* h, long* chunk, unsigned* size);   /* sub-block length (-1: unbounded), ring size */
int hz_dly_set_split(hz_dly* h, int mode);                 /* 0 auto, 1 workgroup per line, 2 launch per sub-block */
int hz_dly_set_stream(hz_dly* h, void* hip_stream);
int hz_dly_synchronize(hz_dly* h);
int hz_dly_set_target_groups(hz_dly* h, int groups);
int hz_dly_profile(hz_dly* h, int enable);
int hz_dly_profile_read(hz_dly* h, double* ms, long* launches);

/* ---- a Bowl block into a Delaybank (`bowl.fill(buf, n);
 * bank.process(buf, out, n);`, bowl.h:50-63 + delay.h:71-97) in one launch: every output equal to
 * the two calls' (the fill buffer written too) when the Bowl is float, the bank is float with
 * <= 128 lines of <= 8 taps, n <= 8192, 2 n <= the ring size and every live tap reads the current sample
 * (time 0) or one at least n and at most size - n samples old (no sample of the block depends on
 * another); otherwise the two block calls.  Both handles on one stream (set_stream). */
int hz_bowl_fill_delaybank(hz_bowl* bowl, float* d_buffer, hz_dly* bank, void* d_out, size_t bsize, int mix);

/* ---- Fourier / StaticSTFT (src/fourier.h:50-194, src/staticSTFT.h:10-177) ----
 * Fourier(int (*processor)(const complex<double>*, complex<double>*), int N, int laps):
 *   window HZ_WIN_HALFHANN; StaticSTFT(int N, int laps): window HZ_WIN_HANN with
 *   HZ_PROC_STATIC_GATE(100, 0.1).  N a power of two in [4, 8192], 1 <= laps <= N.
 * process_block == n x { write(re[t], im[t]); read(&out_re[t], &out_im[t]); }
 * (fourier.h:102-177); im / out_im may be NULL (zero imaginary input / discarded). */
#define HZ_WIN_HALFHANN 0
#define HZ_WIN_HANN 1
#define HZ_PROC_IDENTITY 0
#define HZ_PROC_STATIC_GATE 1 /* p0 = 100, p1 = 0.1: staticSTFT.h:99-128 */
#define HZ_PROC_GATE_KEEP 2   /* p0 = 625: tests/spectral.cpp:32-72 */
#define HZ_PROC_HILBERT 3     /* tests/SFML/hilbert.cpp:37-49 */
#define HZ_PROC_HOST 4        /* host function pointer, per frame, in frame order */
/* the reference's processor type; complex<double>* passed as interleaved double* */
typedef int (*hz_stft_proc)(const double* in, double* out);
typedef struct hz_stft hz_stft;
int hz_stft_create(int N, int laps, int window, int proc, double p0, double p1, int device, hz_stft** out);
int hz_stft_destroy(hz_stft* h);
int hz_stft_set_processor(hz_stft* h, hz_stft_proc fn);
int hz_stft_process_block(hz_stft* h, const double* re, const double* im, double* out_re, double* out_im, size_t n);
int hz_stft_process_block_device(hz_stft* h, const double* d_re, const double* d_im, double* d_out_re,
                                 double* d_out_im, size_t n);
int hz_stft_frames(hz_stft* h, long* frames, long* samples);
/* Per-sample operator API, exactly the reference's state machine: write(re, im) (fourier.h:
 * 102-128), read(&re, &im) (147-177; long double overlap-add, / the int N*laps/2), in any order
 * and number, and the slot operations forward(i) (FFT in[i] -> middle[i], 130-133), backward(i)
 * (IFFT out[i] -> in[i], 135-138) and process(i) (the processor middle[i] -> out[i], 141-144).
 * The O(2 laps) bookkeeping per sample runs on the host; each slot transform and device
 * processor runs on the GPU (one workgroup per N-point transform).  An object is driven either
 * per sample or by blocks (hz_stft_process_block): the first call decides, the other kind then
 * returns HZ_E_STATE. */
int hz_stft_write(hz_stft* h, double real, double imag);
int hz_stft_read(hz_stft* h, double* real, double* imag);
int hz_stft_forward(hz_stft* h, int slot);
int hz_stft_backward(hz_stft* h, int slot);
int hz_stft_process_slot(hz_stft* h, int slot);
/* Time-range shards (STFT): runs of `block` consecutive frames rotate over
 * `world` ranks; this handle computes frame f iff (f / block) % world == rank.  Its other
 * frames are skipped and add nothing to its overlap-add -- in this call or the later calls a
 * frame's window still overlaps -- so the ranks' outputs sum (RCCL reduce) to the unsharded
 * output for any call sizes.  Every rank still streams the whole input (the frame schedule and
 * the history are the reference's).  world == 1: every frame (the default).  Device
 * processors only: HZ_E_UNSUPPORTED with a host processor (it sees every frame in order --
 * replicas only). */
int hz_stft_set_frame_shard(hz_stft* h, int rank, int world, long block);
/* frames completing within the first `samples` input samples of an (N, laps) engine */
int hz_stft_frames_before(int N, int laps, long samples, long* frames);
int hz_stft_set_stream(hz_stft* h, void* hip_stream);
int hz_stft_synchronize(hz_stft* h);
/* Event timing of the frame and overlap-add kernels.  enable > 1 repeats each block's
 * (idempotent) device-processor frame launch `enable` times between the events, so the
 * event overhead is amortised; profile_read then reports frame_ms per single launch. */
int hz_stft_profile(hz_stft* h, int enable);
int hz_stft_profile_read(hz_stft* h, double* frame_ms, double* ola_ms, long* blocks);

/* ---- Cosine (src/fourier.h:197-234): Cosine(int N, double** in, double** out) ----
 * forward = FFTW REDFT10 in -> out (DCT-II, unnormalised), backward = REDFT01 out -> in
 * (DCT-III); the round trip is 2N x identity.  The buffers are pinned host memory owned
 * by the handle.  N a power of two in [4, 8192]. */
typedef struct hz_dct hz_dct;
int hz_dct_create(int N, int device, hz_dct** out);
int hz_dct_destroy(hz_dct* h);
int hz_dct_buffers(hz_dct* h, double** in, double** out);
int hz_dct_forward(hz_dct* h);
int hz_dct_backward(hz_dct* h);
int hz_dct_forward_device(hz_dct* h, const double* d_in, double* d_out, int batch);
int hz_dct_backward_device(hz_dct* h, const double* d_in, double* d_out, int batch);

/* ---- Granulator<double> (src/granulator.h:12-127) reading a Buffer<double> source
 * (src/buffer.h:9-86) through the FUNCTIONAL hann window (src/wave.h:148).
 * Granulator(Wave* window = &hann, Buffer* source (size buffer_size), bool realtime,
 * uint polyphony = 512).  The handle owns the source ring on the device.  One processed
 * sample is the tests/granny.cpp:34-56 loop body:
 *     source.write(in[i]); out[i] = granny(); <requests at i>; source.tick(); granny.tick();
 * A request {at = i, ...} in hz_gran_process is made after the read of sample i (ticks 1
 * at its first read).  hz_gran_request between calls is made after the last processed
 * sample's read and, with ticked = 0, after its tick (ticks 0 at its first read) or, with
 * ticked = 1, before it (the per-sample order operator(); request(); tick()).  Voice
 * allocation is the reference's (first inactive voice; -1 when none is free or size == 0). */
typedef struct hz_gran hz_gran;
typedef struct {
    long at;                                    /* sample index in the call, ascending */
    double offset, size, speed, gain, pan;      /* granulator.h:51 (seconds, ratio, gain) */
} hz_grain_req;
int hz_gran_create(unsigned polyphony, unsigned buffer_size, int device, hz_gran** out);   /* 28-48 */
int hz_gran_destroy(hz_gran* h);
int hz_gran_request(hz_gran* h, double offset, double size, double speed, double gain, double pan, int ticked,
                    int* voice);                                                          /* 51-79 */
/* host pointers, synchronous; voices[k] receives request k's voice (may be NULL) */
int hz_gran_process(hz_gran* h, const double* in, double* out, size_t n, const hz_grain_req* reqs, int nreq,
                    int* voices);
/* device in/out, asynchronous on the handle's stream (requests and voices stay on the host) */
int hz_gran_process_device(hz_gran* h, const double* d_in, double* d_out, size_t n, const hz_grain_req* reqs,
                           int nreq, int* voices);
/* one sample, `source.write(x); y = granny(); granny.tick();` (tests/granny.cpp:36-56), through
 * the device's per-sample server (no launch per sample); the same arithmetic as hz_gran_process */
int hz_gran_sample(hz_gran* h, double x, double* y);
int hz_gran_activity(hz_gran* h, unsigned* activity);   /* active voices; idle() 106-109 is == 0 */
int hz_gran_set_stream(hz_gran* h, void* hip_stream);
int hz_gran_synchronize(hz_gran* h);
int hz_gran_profile(hz_gran* h, int enable);
int hz_gran_profile_read(hz_gran* h, double* ms, long* launches, long* grain_samples);

/* ---- Freezer<N> (src/fourier.h:389-562) with FFrame / IFrame / DFrame (236-387) ----
 * Freezer(laps, width) for N a power of two in [4, 8192].  hz_frz_process runs
 * n x operator()(in[i]) (write; frozen ? slot sum / N : Delay(N)); an event
 * {at, HZ_FRZ_FREEZE | HZ_FRZ_UNFREEZE} is the freeze() / unfreeze() call made before
 * sample `at` (0 <= at <= n, ascending).  The frame choice draws std::rand() on the host,
 * in the reference's order, so srand() seeds both alike. */
#define HZ_FRZ_UNFREEZE 0
#define HZ_FRZ_FREEZE 1
typedef struct hz_frz hz_frz;
typedef struct {
    long at;
    int kind;
} hz_frz_event;
int hz_frz_create(int N, int laps, double width, int device, hz_frz** out);   /* 395-427 */
int hz_frz_destroy(hz_frz* h);
int hz_frz_freeze(hz_frz* h);                                                  /* 468-479 */
int hz_frz_unfreeze(hz_frz* h);                                                /* 481-485 */
int hz_frz_process(hz_frz* h, const double* in, double* out, size_t n, const hz_frz_event* ev, int nev);
int hz_frz_process_device(hz_frz* h, const double* d_in, double* d_out, size_t n, const hz_frz_event* ev, int nev);
int hz_frz_info(hz_frz* h, int* stride, int* frames, int* frozen);
int hz_frz_set_stream(hz_frz* h, void* hip_stream);
int hz_frz_synchronize(hz_frz* h);
/* HIP-event timing of the output kernel (frz_out_kernel) launches while enabled */
int hz_frz_profile(hz_frz* h, int enable);
int hz_frz_profile_read(hz_frz* h, double* ms, long* launches);

/* ---- Filterbank with per-sample coefficient streams ----
 * Subtractive ALLINONE / ONEPERVOICE (src/subtractive.h:215-228, 300-317) retune every band
 * between samples.  hz_fb_process_tv runs n samples with row t of `stream` holding the
 * coefficients in effect at sample t (the staged coefficients are ignored; afterwards the
 * stream's last row is the staged set, as after the reference's last coefficients() call):
 *   HZ_FB_TV_COEFFS    stream [n][2*order+1][N]: forward (order+1) then back (order), band-minor
 *   HZ_FB_TV_RESONANT  stream [n][N] frequencies in Hz, order 2 only: {g, 0, -g},
 *                      {-2 R cos(2 PI f / SR), R^2}, g = resonant(f, R) (subtractive.h:240-249),
 *                      R = param.
 * Smoothers (boost / mix targets), distortion and state are the handle's, shared with
 * hz_fb_process.  _device takes device pointers (asynchronous on the handle's stream). */
#define HZ_FB_TV_COEFFS 0
#define HZ_FB_TV_RESONANT 1
int hz_fb_process_tv(hz_fb* h, const double* in, double* out, size_t n, int kind, const double* stream,
                     double param);
int hz_fb_process_tv_device(hz_fb* h, const double* d_in, double* d_out, size_t n, int kind,
                            const double* d_stream, double param);

/* ---- heterodyne bank chain of tests/harmbank.cpp:77-101, fused over `channels` ----
 * Per sample x:  y = limiter(dry x + gain mixdown(demodulators(synthesis(),
 *     smoothbank(latchbank(&rmsbank, slidebank(modulators(x, analysis())))))))
 * then analysis / synthesis / slidebank / smoothbank / rmsbank tick, with
 *   Oscbank analysis, synthesis   src/oscbank.h:37-68  (two banks: HZ_HET_ANALYSIS, _SYNTHESIS)
 *   Slidebank(order, radii)       src/slidebank.h:60-175 (order <= 8; radii: 2 x channels, re/im)
 *   RMSbank(width)                src/rmsbank.h:29-66
 *   Latchbank(thresh, ratio)      src/latchbank.h:34-85 (the (RMSbank*, signal) form)
 *   Stickbank(stick_order, rad)   src/stickbank.h:44-190 (stick_order <= 4)
 *   Mixer, limiter                src/mixer.h:30-33, src/wave.h:150
 * The oscillator banks start closed at phase 1 with frequency 1 (setOnes); freqmod /
 * activate / open replace Oscbank::freqmod and Multichannel::activate/deactivate/open/close. */
#define HZ_HET_ANALYSIS 0
#define HZ_HET_SYNTHESIS 1
/* hz_het_state: what -> layout (channel-major, doubles) */
#define HZ_HET_STATE_ANALYSIS 0    /* [channels][2] phasors */
#define HZ_HET_STATE_SYNTHESIS 1   /* [channels][2] */
#define HZ_HET_STATE_SLIDE 2       /* [channels][order][2] stage outputs */
#define HZ_HET_STATE_RMS 3         /* [channels] running sums of |s|^2 */
#define HZ_HET_STATE_LATCH 4       /* [channels][2] armed, engaged (0 / 1) */
#define HZ_HET_STATE_STICK 5       /* [channels][stick_order][2] outputs y[t-1-k] */
#define HZ_HET_STATE_HISTORY 6     /* [channels][width] |s|^2, newest first */
typedef struct hz_het hz_het;
int hz_het_create(int channels, int order, const double* radii, double thresh, double ratio, unsigned width,
                  int stick_order, double stick_rad, double dry, double gain, int device, hz_het** out);
int hz_het_destroy(hz_het* h);
int hz_het_setup(hz_het* h, int order, const double* radii);                     /* slidebank.h:63-100 */
int hz_het_freqmod(hz_het* h, int bank, const int* index, const double* hz, int count);   /* oscbank.h:49-56 */
int hz_het_activate(hz_het* h, int bank, const int* index, int count, int on);  /* multichannel.h */
int hz_het_open(hz_het* h, int bank, int on);                                    /* open() / close() */
int hz_het_process(hz_het* h, const double* in, double* out, size_t n);
int hz_het_process_device(hz_het* h, const double* d_in, double* d_out, size_t n);
int hz_het_state(hz_het* h, int what, double* dst);
int hz_het_set_stream(hz_het* h, void* hip_stream);
int hz_het_synchronize(hz_het* h);
int hz_het_profile(hz_het* h, int enable);
int hz_het_profile_read(hz_het* h, double* ms, long* launches, long* channel_samples);

#ifdef __cplusplus
}
#endif
#endif

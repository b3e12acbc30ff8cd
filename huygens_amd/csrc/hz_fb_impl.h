// hz_fb_impl.h -- private header shared by the two Filterbank<double> translation units:
//   hz_filterbank.hip  general engine (time-varying smoothers, distortion functors) + C ABI
//   hz_fb_lti.hip      converged ("LTI") engine
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "hz_common.h"

namespace hz_fbi {

constexpr int kMaxOrder = 4;
constexpr int kLtiGeomChunk128 = 3;   // hz_fb_lti.hip kLtiGeoms: chunk 128 (8192-sample tiles)
constexpr int kStreamBlock = 1024;    // hz_fb_stream.hip: the streaming engine's call length

// MODE_MIX: full pass (mixdown) over one time segment (blockIdx.y) of one band group
//   (blockIdx.x).
// MODE_SEGEND: zero-state end state of each segment but the last (no mixdown), feeding a
//   per-band carry kernel when the bank is too small to fill the chip with bands alone
//   (e.g. 512-band shards on 8 GPUs).
// MODE_STATE (converged engine only): chunk start states x gain of every band to HBM, for the
//   bank-wide correction GEMM (hz_fb_lti.hip, fb_lti_gemm_kernel) instead of a per-group mix.
enum { MODE_MIX = 0, MODE_SEGEND = 1, MODE_STATE = 2 };

// Scalar (SGPR) copy of a wave-uniform double.
__device__ __forceinline__ double uniform(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffff));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// DPP lane moves on a double (two 32-bit halves).  bound_ctrl: lanes whose
// source is outside the pattern read 0.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kDppRowShr = 0x110;   // row_shr:n = 0x110 + n (within 16-lane rows)
// (wave-wide DPP shifts / row_bcast do not exist on CDNA; cross-row moves use
//  ds_bpermute or v_readlane)

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

}  // namespace hz_fbi

constexpr int kMaxOrderRt = 4;   // (= hz_fbi::kMaxOrder)

// ---------------------------------------------------------------------------
// handle (the opaque hz_fb of include/huygens_hip.h)
// ---------------------------------------------------------------------------
struct hz_fb {
    // entry points that touch the staged parameters or the state hold it (setters may come from
    // another thread while samples run: tests/filterbank.cpp:217-252 vs 200-210)
    std::recursive_mutex mu;
    // setters waiting for `mu`: a per-sample call lets them in first (a thread calling operator()
    // in a tight loop would otherwise re-take the lock before a waiting setter is scheduled)
    std::atomic<int> setter_wait{0};
    long pg_gen = 0, coef_gen = 0;   // generations of the staged targets / coefficients
    long long setter_seq = 0;        // per-sample calls served when the last setter ran
    int order = 2, N = 0, N_total = 0, band_begin = 0, device = 0;
    double sp = 0, sg = 0;
    int rec = 8;
    // host shadows of the staged parameters
    std::vector<double> F, B, pin, gin;
    bool dirty_coef = true, dirty_pin = true, dirty_gin = true;
    int dist_id = HZ_DIST_NONE;
    double dist_param = 0;
    // geometry
    int waves = 16, bands_per_wave = 1;
    // device buffers
    double *d_rec = nullptr, *d_pin = nullptr, *d_gin = nullptr;
    double *d_ystate[2] = {nullptr, nullptr}, *d_pg[2] = {nullptr, nullptr};
    int scur = 0;  // current state buffer (ping-pong per launch)
    double* d_xhist[2] = {nullptr, nullptr};
    int xcur = 0;
    // the reference's rings hold O+1 rows; the row the engine state (O rows) leaves out sits in
    // d_ystate[scur ^ 1][.][O-1] / d_xhist[xcur ^ 1][O-1] after a 1-sample call or a tick
    // (hz_fb_tick), and is not kept after longer calls
    bool spare_ok = true;
    // plan of the last LTI launch (hz_fb_lti_plan): time segments, prepass tiles skipped per
    // segment (horizon), fine prepass parts per segment
    long plan_nseg = 0, plan_skip_tiles = 0;
    int plan_fine = 0, plan_chunk = 0;
    double* d_partial = nullptr;
    size_t partial_cap = 0;  // doubles
    double* d_seg = nullptr;  // segment start states
    size_t seg_cap = 0;
    int target_groups = 256;  // workgroups wanted per launch (CU count)
    double *d_in = nullptr, *d_out = nullptr;
    size_t io_cap = 0;       // doubles
    // host-buffer calls that take the streaming engine: pinned, device-mapped staging the kernel
    // reads and writes directly ([kStreamBlock] in, then [kStreamBlock] out)
    double* pin_io = nullptr;   // + 128 completion flags (long long) after the in/out blocks
    long long pin_seq = 0;
    std::vector<double> h_rec;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // profiling
    bool prof = false;
    std::vector<hipEvent_t> ev;  // quintuplets: start, mix start, mix end, reduce start, reduce end
    size_t ev_used = 0;
    // per quintuplet: bit 1 = mix start not recorded (same point as start), bit 3 = reduce
    // start not recorded (same point as mix end); every record costs a few us of GPU time
    std::vector<unsigned char> ev_skip;
    // per quintuplet: launches per timed kernel between its events (hz_fb_profile(h, rep > 1): the
    // stationary engine's idempotent kernels repeated back to back, so one event pair's own
    // latency is spread over rep launches)
    std::vector<unsigned char> ev_rep;
    int prof_rep = 1;
    long prof_launches = 0;
    // converged (LTI) path, hz_fb_lti.hip
    int path_mode = HZ_FB_PATH_AUTO;
    int last_path = HZ_FB_PATH_GENERAL;
    int lti_geom = -1;               // index into kLtiGeoms (hz_fb_lti.hip); -1 = by call length
    struct LtiRecSet {               // LTI records + Fmix per chunk length (geometry)
        bool dirty = true;           // coefficients changed since the records were built
        bool fmix_valid = false;     // Fmix matches the current coefficients, pin and gin
        int rs = 0;                  // record size (doubles)
        double* d_rec = nullptr;
        size_t cap = 0;
        double* d_fmix = nullptr;    // [L][L+O]
        double* d_kt = nullptr;      // [N O padded to 4][L] homogeneous responses (correction GEMM)
        size_t kt_cap = 0;
        long horizon = -2;           // samples after which ||M^k|| < 2^-64 for every band
                                     // (-1: none within 2^18; -2: not computed yet)
    };
    static constexpr int kLtiSets = 4;   // chunks 16, 32, 64, 128
    LtiRecSet lti_set[kLtiSets];
    std::vector<double> pg_host;     // host mirror of the smoother state [N][2] (pre, gain)
    long mirror_clock = 0;           // samples processed (the closed form is applied lazily)
    std::vector<long> mirror_at;     // [N] mirror_clock at which pg_host[b] was last brought current
    bool converged = false;          // pg_host at the targets; cleared by every setter
    // LTI launches are split in chunks whose cross-group reduce runs on a second stream,
    // overlapped with the next chunk's mix kernel (double-buffered partial slab)
    hipStream_t stream_red = nullptr;
    std::vector<hipEvent_t> sync_ev;  // ordering events (no timing)
    double* d_xhist_red = nullptr;    // x history at the call start, for the first chunk's reduce
    // a coefficient-stream call leaves its last row staged as the coefficients; the row is
    // copied back asynchronously and turned into F/B only when they are next needed
    double* tv_row = nullptr;         // pinned host copy of the stream's last row
    size_t tv_row_cap = 0;            // doubles
    hipEvent_t tv_ev = nullptr;       // the copy's completion
    bool tv_pending = false;
    int tv_kind = 0;
    double tv_param = 0;
    // stationary engine (hz_fb_resp.hip): the bank response h of the converged bank and the last
    // K inputs, from which the band states follow once the bank has been stationary for K samples
    struct Resp {
        int mode = HZ_FB_RESP_EAGER;     // HZ_FB_RESP_OFF / _EAGER / _LAZY
        long K = -2;                     // horizon (samples, multiple of 8192, 2^-53); -1 none; -2 unknown
        bool h_valid = false;            // d_h / d_H match F, B, pin, gin
        long run = 0;                    // converged samples in a row written into the history
        bool implicit = false;           // LAZY: ystate[scur] not yet materialised from the history
        long calls = 0;                  // stationary calls made
        long min_call = 0;               // shortest stationary / history-keeping call (0: 16384)
        long bands_per_sample = -1;      // cost model: stationary when N n >= this (K + n) (-1: 256)
        // time-range shards (multi-GPU): the whole bank's response, summed over the band shards by
        // the caller (hz_fb_set_bank_response; cleared by every setter), and this rank's share
        std::vector<double> h_over;
        bool over_valid = false;
        int shard_rank = 0, shard_world = 1;
        // outside its share a time-sharded call writes zeros (1, default: the ranks' outputs sum to
        // the call's mix) or leaves the output untouched (0: disjoint shares, nothing to reduce)
        bool shard_zero = true;
        // a time-sharded handle takes the stationary engine only when the caller has armed it on
        // every rank (hz_fb_arm_time_shard after an all-reduce of hz_fb_stationary_ready), so all
        // ranks switch engines in the same call; cleared by every setter
        bool armed = false;
        double* d_hist[2] = {nullptr, nullptr};   // [K] last K inputs (ping-pong)
        size_t hist_cap0 = 0, hist_cap1 = 0;
        int hcur = 0;
        double* d_h = nullptr;           // [K] aggregate impulse response
        size_t h_cap = 0;
        double* d_hpart = nullptr;       // [64-band groups][K]
        size_t hpart_cap = 0;
        double* d_coef = nullptr;        // F [N][O+1], B [N][O]
        size_t coef_cap = 0;
        double* d_H = nullptr;           // [Qp][2048] complex partition spectra, then [Qp] bin 2048
        size_t H_cap = 0;
        double* d_Z = nullptr;           // [rows][2048] complex window spectra, then [rows] bin 2048
        size_t Z_cap = 0;
        double* d_Y = nullptr;           // [B][2048] complex output spectra
        size_t Y_cap = 0;
        double* d_tw = nullptr;          // W_4096^k, k < 2048 (complex)
        // column-split path (hz_fb_col.h): W_4096^k for k < 4096, H in column layout, the inverse
        // columns T of a call, the combine's column map
        bool col_on = false;             // hz_fb_tune_response_engine (column split: opt-in)
        int last_engine = 0;             // 0 three-kernel, 1 column-split (last stationary call)
        double* d_tw4k = nullptr;
        double* d_Hc = nullptr;
        size_t Hc_cap = 0;
        double* d_T = nullptr;
        size_t T_cap = 0;
        unsigned char* d_cmap = nullptr;
        double* d_sop = nullptr;         // band-state pass: pin E operands (fb_state_prepare)
        size_t sop_cap = 0;
        double* d_spart = nullptr;       // band-state pass: segment partials, arrival counters
        size_t spart_cap = 0;
        unsigned* d_scount = nullptr;
        size_t scount_cap = 0;
        double* d_zero = nullptr;        // N O zeros (x history / start of the zero-start pass)
        size_t zero_cap = 0;
        // modal band states (hz_fb_modal.h): banks whose poles sit on one circle on the 2 pi / 8192
        // grid get their states from a fold and one DFT instead of the MFMA pass
        bool modal_on = true;            // hz_fb_tune_modal
        bool modal_ok = false;           // the current bank qualifies (built with d_h)
        bool modal_last = false;         // the last stationary call used it
        double* d_mpar = nullptr;        // BandPar [N]
        size_t mpar_cap = 0;
        double* d_mtab = nullptr;        // R_g^r [8192], R_g^(8192 s) [S], e^(2 pi i q / 8192) [8192]
        size_t mtab_cap = 0;
        double* d_mA = nullptr;          // [2][64][128] complex (phase 1 -> phase 2)
        size_t mA_cap = 0;
        double* d_mexc = nullptr;        // exceptional responses [nexc][K + 1], then their partials
        size_t mexc_cap = 0;
        int* d_mint = nullptr;           // csr_ptr [65], csr (band, k2) [N], exceptional bands [8]
        size_t mint_cap = 0;
        int mexc_n = 0, mexc_chunks = 0, mS = 0;
        long h_gen = 0;                  // d_h rebuilds (the streaming spectra follow it)
        // streaming calls (hz_fb_stream.hip): 1024-sample blocks of a stationary bank, one launch
        // each, through a frequency-domain delay line; the history in a mirrored ring
        struct Stream {
            bool on = true;              // engine enabled (hz_fb_tune_stream)
            long R = 0;                  // ring length (K + 2048); the ring holds 2 R doubles
            double* d_line = nullptr;    // [2 R]: sample of position i at i mod R and i mod R + R
            size_t line_cap = 0;
            long pos = 0;                // samples written; the history is positions [pos - K, pos)
            bool line_hist = false;      // the history lives in the ring (not resp.d_hist)
            bool fdl_valid = false;      // d_ZS holds the spectra of the windows ending at pos
            long hs_gen = -1;            // h_gen the partition spectra were built from
            int head = 0;                // slot of the next call's window
            double *d_ZS = nullptr, *d_HS = nullptr;   // [K/1024][33][32] complex
            size_t zs_cap = 0, hs_cap = 0;
            double* d_CR = nullptr;      // [2][33][32] tail columns C, then [2][33][32] MAC sums R (complex)
            long blk = 0;                // streamed blocks since the ring was primed (parity of C / R)
            double* d_tw = nullptr;      // twiddles (W_64, W_32, W_2048)
            long pend = 0;               // streamed samples not yet applied to the smoothers / x history
            long calls = 0;
            long long* flags_dev = nullptr;   // completion flags of a host-buffer call (hz_fb_process)
            long long flags_seq = 0;
            // horizons past the head (K > 2^17, e.g. R = 0.9999): the response's tail h[K1, K) is
            // convolved per 16384-sample epoch ahead of time, on a side stream, by the long-call
            // engine's kernels (hz_fb_resp.hip fb_resp_tail_conv); blocks add tail_out
            bool tail = false;
            long K1 = 0;                 // head horizon (<= 2^17)
            int tQ = 0;                  // tail partitions of 2048
            double* d_tH = nullptr;      // [tQp][2048] complex tail partition spectra, then [tQp] bin 2048
            size_t tH_cap = 0;
            double *d_tZ = nullptr, *d_tY = nullptr;   // the tail convolution's window / output spectra
            size_t tZ_cap = 0, tY_cap = 0;
            double* d_tout = nullptr;    // [2][16384] tail outputs of epochs e (slot e & 1)
            size_t tout_cap = 0;
            long tail_launched = -1;     // last epoch whose tail convolution was issued
            bool tail_async[2] = {false, false};   // that slot's convolution ran on the side stream
            hipStream_t side = nullptr;
            hipEvent_t ev_main = nullptr, ev_tail[2] = {nullptr, nullptr};
            // gain transients (round 6): mix() while streaming keeps the engine.  The gain smoothers
            // share s_g, so g_n(t) = gin_n + s_g^(t - dref) D_n and the mix is
            //     out(t) = conv(h, x)(t) + s_g^(t - dref) conv(h_D, x)(t),  h_D = sum_n D_n r_n,
            // both responses updated per setter from the per-band responses r_n (resident in HBM,
            // [K][N]); a second launch per block (the D pass) adds the transient term
            bool dmode = false;
            long dref = 0;               // stream position the D term is referred to
            double dmax = 0;             // bound on max |D_n| at dref (decay check)
            double gin_max = 0;          // max |gin_n| (the decay check's scale)
            long dsetters = 0;           // setters applied as transients
            double* d_hD = nullptr;      // [K1] h_D
            size_t hD_cap = 0;
            double* d_HSD = nullptr;     // [K1/1024 + 8][33][32] its spectra
            size_t hsd_cap = 0;
            double* d_CRD = nullptr;     // its C / R parities
            // r_n (pre = pin, no gain) in partition form (hz_fb_stream.hip stream_rbasis_kernel)
            double* d_r0 = nullptr;      // [N][1024] partition 0
            double* d_phi = nullptr;     // [N][O][1024] homogeneous basis responses
            double* d_st = nullptr;      // [N][Q][O] states at the partition starts
            double* d_rsp = nullptr;     // [N][O + 1][33][32] double2: spectra of r0, phi
            size_t r0_cap = 0, phi_cap = 0, st_cap = 0, rsp_cap = 0;
            bool rband_valid = false;
            double* d_sgpow = nullptr;   // s_g^j, j < 1024
            double sgpow_of = -1;        // the s_g it holds
            std::vector<double> h_delta;   // the last setter's bands
            unsigned long long* d_trace = nullptr;   // (diagnostic, HZ_STREAM_TRACE) launch timelines
            int trace_n = 0, trace_kind[1024] = {}, trace_wg[1024] = {};
            std::vector<double> gin_base;   // the gins d_h is built with
            bool prime_main = false;     // C / R of the main pass to recompute (h changed, ring valid)
            bool prime_d = false;        // ... of the D pass
        } st;
    } resp;
    // per-sample path (hz_fb_rt.hip): OP_FB requests to the device's per-sample server (hz_rt.hip)
    struct Rt {
        bool active = false;         // the state is in the per-sample layout (ring rows)
        bool computed = false;       // the reference's `computed` (filterbank.h:127-128, 168)
        bool spare_known = false;    // the ring row at origin is known (after any compute)
        long long seq = 0;           // samples served
        long pending_ticks = 0;      // tick() calls since the last served request
        double cached = 0;           // the last served sample
        int cached_dist = 0;
        double xr[kMaxOrderRt + 1] = {};   // input ring (ring order), host mirror
        long pg_gen = 0, coef_gen = 0;     // generations the server's arrays hold
        // one-band target setters since the server's copy (generation sp_base .. sp_gen): the next
        // sample sends (band, pin, gin) triples instead of both [N] arrays while the list covers
        // every target change since (sp_base == pg_gen, sp_gen == the handle's pg_gen)
        std::vector<int> dirty;
        std::vector<unsigned char> mark;   // [N] band in `dirty`
        long sp_base = 0, sp_gen = 0;
        double* pin1 = nullptr;      // pinned staging (x history, a cached sample)
        double* d_coef = nullptr;    // [N][2O+1] coefficients, then [N][O+1] ring rows
        size_t coef_cap = 0;
        std::vector<double> h_coef;
        bool many = false;           // the server last served these rows through OP_FB_MANY
    } rt;
};

namespace hz_fbi {

inline void cpu_relax() { __builtin_ia32_pause(); }

// bounded spins before a blocking wait: a thread put to sleep on the mutex costs the other side a
// scheduler wake-up (5-10 us) per hand-off, a quarter of a sample period at 48 kHz
constexpr int kSpinSetter = 1 << 16;    // ~ a few ms of pause instructions
constexpr int kSpinSample = 1 << 20;

// the hold of a setter or any other entry point but operator() / tick() (SampleLock), announced
// from before it locks until after it unlocks, so a per-sample call neither takes the lock ahead
// of it (an audio thread spinning on the lock would otherwise starve a blocked waiter) nor blocks
// behind it (hz_fb::setter_wait); it spins for the lock while a sample is being served
struct HandleLock {
    hz_fb* h;
    explicit HandleLock(hz_fb* h_) : h(h_) {
        h->setter_wait.fetch_add(1);
        int spin = 0;
        while (!h->mu.try_lock()) {
            if (++spin == kSpinSetter) {
                h->mu.lock();
                break;
            }
            cpu_relax();
        }
    }
    ~HandleLock() {
        h->mu.unlock();
        h->setter_wait.fetch_sub(1);
    }
};

// a per-sample call's hold (operator() / tick()): announced setters go first (this sample sees
// them) for at most kAnnounceWaitNs -- a setter thread descheduled between its announcement and
// the lock must not stall the audio thread for a scheduler slice -- then the lock, spinning
// rather than sleeping on the mutex
constexpr long long kAnnounceWaitNs = 20000;
struct SampleLock {
    hz_fb* h;
    explicit SampleLock(hz_fb* h_) : h(h_) {
        if (h->setter_wait.load(std::memory_order_acquire) > 0) {
            const auto t0 = std::chrono::steady_clock::now();
            for (int spin = 1; h->setter_wait.load(std::memory_order_acquire) > 0; ++spin) {
                if ((spin & 63) == 0 && std::chrono::duration_cast<std::chrono::nanoseconds>(
                                            std::chrono::steady_clock::now() - t0).count() > kAnnounceWaitNs)
                    break;
                cpu_relax();
            }
        }
        int spin = 0;
        while (!h->mu.try_lock()) {
            if (++spin == kSpinSample) {
                h->mu.lock();
                break;
            }
            cpu_relax();
        }
    }
    ~SampleLock() { h->mu.unlock(); }
};

// hz_filterbank.hip
int fb_set_lds_attr(const void* kernel);
int fb_prof_events(hz_fb* h, hipEvent_t** e);
void fb_mirror_advance(hz_fb* h, long len);  // O(1): the closed form is applied lazily
void fb_mirror_sync(hz_fb* h);               // bring pg_host up to date (before a setter)
void fb_mirror_sync_band(hz_fb* h, int l);   // band l only (before a one-band setter)
// a target setter advances pg_gen: l = its local band, -1 = a band of another shard, kAllBands = all
constexpr int kAllBands = -2;
void fb_rt_target_setter(hz_fb* h, int l);
int fb_launch_general(hz_fb* h, const double* d_in, double* d_out, long n);
int fb_upload_staged(hz_fb* h);              // staged setters -> device
int fb_tv_materialize(hz_fb* h);             // pending stream row -> F/B (hz_fb_tv.hip)
// hz_fb_lti.hip
int fb_lti_geom(const hz_fb* h, long n);  // LTI geometry for a call of n samples
int fb_lti_chunk(int geom);                // samples per lane chunk of a geometry
bool fb_lti_gemm_geom(int geom);           // geometry runs the correction GEMM path
// hz_fb_gemm.hip: part[s][t] = correction of sample t over band-state slice s (chunk 64); picks
// the slice count (<= max_slices, reported in *slices_out)
int fb_lti_gemm_launch(const double* gs, const double* kt, int bs_pad, double* part, long n_pad, int ntiles, int L,
                       int target_groups, int max_slices, hipStream_t stream, int* slices_out);
bool fb_converged(hz_fb* h);
int fb_launch_lti(hz_fb* h, int geom, const double* d_in, double* d_out, long n);
long fb_horizon(const hz_fb* h, int log2_bound);   // samples K with ||M^K|| < 2^log2_bound for every band (-1: > 2^18)
// zero-start band states after the window x[0, len) (len a multiple of 8192) -> out[band][O], on
// stream st: the stationary engine's band-state pass (hz_fb_state.hip)
int fb_state_window(hz_fb* h, const double* x, long len, double* out, hipStream_t st);
int fb_state_prepare(hz_fb* h);   // its records and pin E operands (current coefficients, pin), on h->stream
int fb_lti_prepare_end(hz_fb* h, long len);   // its records for the current coefficients
// hz_fb_resp.hip (stationary engine)
void fb_resp_init(hz_fb* h);
void fb_resp_invalidate(hz_fb* h, bool coefficients);   // targets / coefficients changed
void fb_resp_setter(hz_fb* h);   // any setter, also for bands of other shards: the bank response changes
bool fb_resp_eligible(hz_fb* h, long n, bool conv);   // this handle alone (no arming)
bool fb_resp_time_sharded(const hz_fb* h);            // the engine choice is the caller's (armed)
int fb_launch_resp(hz_fb* h, const double* d_in, double* d_out, long n);
int fb_resp_track(hz_fb* h, const double* d_in, long n, bool conv);  // history after any call
int fb_resp_materialize(hz_fb* h);                                  // LAZY: band states now
void fb_resp_free(hz_fb* h);
int fb_resp_setup(hz_fb* h);   // horizon and history buffers
int fb_resp_build(hz_fb* h);   // + h, its spectra and the band-state operands for the current bank
// hz_fb_stream.hip (streaming calls of a stationary bank)
bool fb_stream_trackable(hz_fb* h, long n, bool conv);   // a call the ring keeps the history of
bool fb_stream_eligible(hz_fb* h, long n, bool conv);    // ... and that streams (history >= K)
int fb_launch_stream(hz_fb* h, const double* d_in, double* d_out, long n);
int fb_stream_workgroups();   // workgroups of one streaming launch (completion flags)
int fb_stream_track(hz_fb* h, const double* d_in, long n, bool conv);   // a short per-band call
int fb_stream_materialize(hz_fb* h);   // band states, smoothers, x history from the ring
int fb_stream_upkeep(hz_fb* h);        // smoothers and x history over the streamed samples
int fb_stream_to_hist(hz_fb* h);       // the ring's history back to resp.d_hist (long calls)
void fb_stream_reset(hz_fb* h);        // state overwritten (set_state, tick)
void fb_stream_free(hz_fb* h);
int fb_stream_gain_setter(hz_fb* h);      // a gin-only setter as a streaming transient (0: not applied,
                                          // 1: applied, d_gin written by its launch)
bool fb_stream_dmode(const hz_fb* h);     // a gain transient is streaming (gains still moving)
void fb_stream_dclear(hz_fb* h);          // leave the transient mode (the response is rebuilt)
// the streaming engine's response tail (hz_fb_resp.hip): partition spectra of h[K1, K), and the
// convolution out[i] = sum_{tau < Kt} h[K1 + tau] u[Kt + i - tau], i < n, of a contiguous u
int fb_resp_tail_spectra(hz_fb* h, long K1);
int fb_resp_tail_conv(hz_fb* h, const double* u, long n, double* out, hipStream_t st);
// hz_filterbank.hip: one ring rotation of a tick() without compute (needs spare_ok)
int fb_tick_rotate(hz_fb* h);
// hz_fb_rt.hip (per-sample engine)
bool fb_rt_supported(const hz_fb* h);
int fb_rt_stop(hz_fb* h);    // the resident kernel leaves (stream-ordered), pending ticks applied
// a block call after operator() without tick(): the reference's loop returns the cached sample
// first (re-mixed with the block's distortion) and ticks; -> samples consumed (0 or 1)
int fb_rt_resolve(hz_fb* h, double* y0);
double* fb_rt_cached_slot(hz_fb* h);   // pinned host double for an async copy of that sample
void fb_rt_free(hz_fb* h);

}  // namespace hz_fbi

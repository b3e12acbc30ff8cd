/*
 * hz_oracle.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Scalar C restatement of the amcerbu/huygens bank hot path, op for op, used
 * as the parity checker for the HIP kernels in huygens_amd/csrc.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: the reference itself cannot be compiled in this image
 * (Eigen >= 3.4, FFTW3, PortAudio and RtMidi headers are absent; see
 * DESIGN.md "Oracle") and its tests hold no golden vectors.  This
 * restatement is therefore pinned against (a) an independent numpy
 * restatement that writes tests/golden/ fixtures, (b) scipy.signal.lfilter /
 * numpy.fft / scipy.fft.dct known-answer checks of the third-party maths
 * (Eigen GEMV, FFTW DFT/REDFT conventions), and (c) closed-form known
 * answers.  Strictly, by the reference's own fixtures: parity unpinned.
 *
 * Constants follow /root/reference/src/includes.h:30-48 (truncated PI,
 * integer SR, relaxation()).
 */
#ifndef HZ_ORACLE_H
#define HZ_ORACLE_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

double orc_relaxation(double k);
double orc_mtof(double m);
double orc_ftom(double f);

/* ---- Filterbank<double> (src/filterbank.h:16-188) ---------------------- */
typedef struct orc_fb orc_fb;
orc_fb* orc_fb_create(int order, int N, double k_p, double k_g);
void    orc_fb_destroy(orc_fb* fb);
void    orc_fb_coefficients(orc_fb* fb, int n, const double* fwd, int nf, const double* back, int nb);
void    orc_fb_boost(orc_fb* fb, int n, double v);
void    orc_fb_boost_all(orc_fb* fb, const double* v, int count);
void    orc_fb_mix(orc_fb* fb, int n, double v);
void    orc_fb_mix_all(orc_fb* fb, const double* v, int count);
void    orc_fb_open(orc_fb* fb);
double  orc_fb_sample(orc_fb* fb, double x, int dist_id, double dist_param);
void    orc_fb_tick(orc_fb* fb);
void orc_fb_get_state(const orc_fb* fb, double* buf);
void    orc_fb_process(orc_fb* fb, const double* in, double* out, long n, int dist_id, double dist_param);
/* per-sample coefficient streams (kind 0: [n][2O+1][N] coefficients; kind 1: [n][N] resonant
 * frequencies, order 2, R = param); see hz_oracle.c */
void    orc_fb_process_tv(orc_fb* fb, const double* in, double* out, long n, int kind, const double* stream,
                          double param, int dist_id, double dist_param);
double  orc_resonant(double frequency, double Q);
void    orc_fb_resonant_coefficients(double frequency, double R, double* fwd, double* back);

/* ---- Oscbank<double,N> (src/oscbank.h:15-97, src/multichannel.h:16-159) */
typedef struct orc_osc orc_osc;
orc_osc* orc_osc_create(int N, double k);
void     orc_osc_destroy(orc_osc* o);
void     orc_osc_freqmod(orc_osc* o, int index, double hz);
void     orc_osc_activate(orc_osc* o, const int* idx, int count);
void     orc_osc_deactivate(orc_osc* o, const int* idx, int count);
void     orc_osc_open(orc_osc* o);
void     orc_osc_close(orc_osc* o);
void     orc_osc_tick(orc_osc* o);
void     orc_osc_mixdown(orc_osc* o, double* re, double* im);
void     orc_osc_phases(orc_osc* o, double* z /* 2N interleaved */);
int      orc_osc_active_count(orc_osc* o);
/* n x { mix[i] = mixdown(); per_band[i][:] = phases; tick(); } (per_band may be NULL) */
void     orc_osc_fill(orc_osc* o, double* mix /* 2n */, double* per_band /* 2nN */, long n);

/* ---- Additive<double> (src/additive.h:11-71 + src/minimizer.h note API) - */
typedef struct orc_add orc_add;
orc_add* orc_add_create(int voices, int overtones, double decay, double harmonicity, double k);
void     orc_add_destroy(orc_add* a);
int      orc_add_request(orc_add* a, double fundamental, double amplitude);
void     orc_add_release(orc_add* a, int voice);
int      orc_add_makenote(orc_add* a, double pitch, double amplitude);
void     orc_add_endnote(orc_add* a, double pitch);
double   orc_add_sample(orc_add* a);
void     orc_add_tick(orc_add* a);
void     orc_add_fill(orc_add* a, double* out, long n);

/* ---- Sinusoids<double> (src/sinusoids.h:10-79) -------------------------- */
typedef struct orc_sin orc_sin;
orc_sin* orc_sin_create(double fundamental, int overtones, double decay, double harmonicity, double k);
void     orc_sin_destroy(orc_sin* s);
void     orc_sin_fundmod(orc_sin* s, double target);
void     orc_sin_decaymod(orc_sin* s, double target);
void     orc_sin_harmmod(orc_sin* s, double target);
double   orc_sin_sample(orc_sin* s);
void     orc_sin_tick(orc_sin* s);
void     orc_sin_fill(orc_sin* s, double* out, long n);

/* ---- Bowl<T> (src/bowl.h:10-74), T = double (is_float 0) or float (1) ---- */
typedef struct orc_bowl orc_bowl;
orc_bowl* orc_bowl_create(int overtones, const double* f, const double* a, const double* d, int count,
                          int is_float);
void      orc_bowl_destroy(orc_bowl* b);
void      orc_bowl_trigger(orc_bowl* b);
void      orc_bowl_seek(orc_bowl* b, long ticks);
int       orc_bowl_fill(orc_bowl* b, float* buffer, long bsize);
void      orc_bowl_render(orc_bowl* b, double* out, long n);

/* ---- Delay<T> / Delaybank<T,N> (src/delay.h:10-108, src/buffer.h:9-86) ---- */
typedef struct orc_dly orc_dly;
orc_dly* orc_dly_create(int lines, unsigned sparsity, unsigned time, int is_float);
void     orc_dly_destroy(orc_dly* b);
void     orc_dly_coefficients(orc_dly* b, int line, const unsigned* ft, const double* fg, int nf,
                              const unsigned* bt, const double* bg, int nb);
void     orc_dly_modulate_forward(orc_dly* b, int line, unsigned n, unsigned t, double g);
void     orc_dly_modulate_back(orc_dly* b, int line, unsigned n, unsigned t, double g);
void     orc_dly_process(orc_dly* b, const void* in, void* out, long n, int in_per_line, int mix);
unsigned orc_dly_origin(orc_dly* b);
void orc_dly_tick(orc_dly* b, unsigned long count);

/* ---- Fourier / StaticSTFT / Cosine (src/fourier.h:50-234, src/staticSTFT.h:10-177) ---- */
#define ORC_PROC_IDENTITY 0
#define ORC_PROC_STATIC_GATE 1   /* p0 = 100, p1 = 0.1 */
#define ORC_PROC_GATE_KEEP 2     /* p0 = 625 */
#define ORC_PROC_HILBERT 3
#define ORC_PROC_CALLBACK 4
typedef int (*orc_stft_cb)(const double* in, double* out);
typedef struct orc_stft orc_stft;
orc_stft* orc_stft_create(int N, int laps, int window, int proc, double p0, double p1);
void      orc_stft_set_callback(orc_stft* s, orc_stft_cb cb);
void      orc_stft_destroy(orc_stft* s);
void orc_stft_forward(orc_stft* s, int i);
void orc_stft_backward(orc_stft* s, int i);
void orc_stft_process_slot(orc_stft* s, int i);
void      orc_stft_write(orc_stft* s, double re, double im);
void      orc_stft_read(orc_stft* s, double* re, double* im);
void      orc_stft_process_block(orc_stft* s, const double* re, const double* im, double* out_re,
                                 double* out_im, long n);
long      orc_stft_frames(orc_stft* s);
void      orc_dft(const double* x, double* y, int N, int sign);
void      orc_dct(const double* x, double* y, int N, int kind);

/* ---- Granulator<double> (src/granulator.h:12-127) over Buffer<double> (src/buffer.h) ---- */
typedef struct orc_gran orc_gran;
orc_gran* orc_gran_create(unsigned polyphony, unsigned buffer_size);
void      orc_gran_destroy(orc_gran* g);
int       orc_gran_request(orc_gran* g, double offset, double size, double speed, double gain, double pan);
void      orc_gran_write(orc_gran* g, double x);
double    orc_gran_sample(orc_gran* g);
void      orc_gran_tick(orc_gran* g);
unsigned  orc_gran_activity(orc_gran* g);
/* n x { write(in[i]); out[i] = sample(); requests k with at[k] == i, in order (req: 5
 * doubles offset, size, speed, gain, pan; voices[k] = returned voice); tick(); }  (at sorted) */
void      orc_gran_process(orc_gran* g, const double* in, double* out, long n, const long* at, const double* req,
                           int nreq, int* voices);

/* ---- Freezer<N> / FFrame / IFrame / DFrame (src/fourier.h:236-562) ---------- */
typedef struct orc_frz orc_frz;
orc_frz* orc_frz_create(int N, int laps, double width);
void     orc_frz_destroy(orc_frz* z);
int      orc_frz_geometry(orc_frz* z, int* stride, int* M);   /* returns size = M * stride */
void     orc_frz_freeze(orc_frz* z);
void     orc_frz_unfreeze(orc_frz* z);
int      orc_frz_frozen(orc_frz* z);
double   orc_frz_sample(orc_frz* z, double sample);
/* n x { events k with at[k] == i (kind 1 freeze, 0 unfreeze), in order; out[i] = sample(in[i]) } */
void     orc_frz_process(orc_frz* z, const double* in, double* out, long n, const long* at, const int* kind, int nev);

/* ---- heterodyne chain (tests/harmbank.cpp:77-101): Oscbank x2, Modbank, Slidebank, RMSbank,
 * Latchbank, Stickbank, Mixer, limiter ---- */
typedef struct orc_het orc_het;
orc_het* orc_het_create(int N, int order, const double* radii, double thresh, double ratio, unsigned width,
                        int stick_order, double stick_rad, double dry, double gain);
void     orc_het_destroy(orc_het* h);
void     orc_het_setup(orc_het* h, int order, const double* radii);        /* Slidebank::setup */
void     orc_het_freqmod(orc_het* h, int bank, int index, double hz);      /* bank 0 analysis, 1 synthesis */
void     orc_het_activate(orc_het* h, int bank, const int* idx, int count, int on);
double   orc_het_sample(orc_het* h, double x);
void     orc_het_process(orc_het* h, const double* in, double* out, long n);
/* state readback in the layouts of hz_het_state (include/huygens_hip.h) */
void     orc_het_state(orc_het* h, int what, double* dst);

/* distortion functors (tests/filterbank.cpp:158-176, src/wave.h:150) */
double orc_dist(int id, double v, double param);

#ifdef __cplusplus
}
#endif
#endif

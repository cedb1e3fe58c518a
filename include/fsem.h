/*
 * fsem.h -- C-ABI of libfsem.so, the MI355X (gfx950) engine behind
 * fast_speech_enhancement_metrics_amd.PESQ / .STOI.
 *
 * The reference (kcoost/fast_speech_enhancement_metrics) is a pure-Python/PyTorch
 * library with no FFI layer; its drop-in boundary is the metric class API
 *   BaseMetric.__call__(clean, denoised) -> list[dict]      fast_se_metrics/base.py:41-43
 * Each entry point below replaces the reference computation named next to it; the
 * Python host layer (fast_speech_enhancement_metrics_amd/base.py, PESQ.py, STOI.py) keeps
 * the reference's class API and calls these through ctypes.
 *
 * Conventions
 *  - every pointer argument is DEVICE memory owned by the caller (torch tensors);
 *  - the library allocates nothing: scratch space comes from `ws` (size from the
 *    matching *_workspace_bytes query); work is enqueued asynchronously on `stream`
 *    (a hipStream_t; NULL = the default stream) and the call returns immediately;
 *  - signals are float32 rows: element (b, t) of a batch lives at ptr[b * ld + t]; the
 *    PESQ and STOI entries read rows in 16-byte pieces, so each row must be readable up to
 *    ceil4(length) floats (values past `length` are never used);
 *  - per-row lengths (variable-length batches): the PESQ and STOI entries take
 *    `lengths`, a DEVICE int32[batch] array or NULL.  NULL means every row has `length`
 *    samples.  Otherwise row b holds lengths[b] samples (clamped to [0, length]; `length`
 *    is then the row capacity, sizing workspace and layouts) and its result is that of the
 *    reference called on the unpadded row alone; rows too short for the metric give NaN
 *    (instead of FSEM_ESHORT, which only the whole-batch form returns);
 *  - rows are at most 2^29 samples long (9.3 h at 16 kHz), before and after any resampling:
 *    the kernels address rows with 32-bit byte offsets; longer rows give FSEM_EINVAL;
 *  - input domain (tests/test_edges_ref_gpu.py against the reference's own outputs,
 *    tests/golden/edges_16k.npz, tone_probe_10k.npz, lowpass_10k.npz; every figure below is
 *    per row, profiles/r4_g/edges_rows.log):
 *      PESQ: any finite scale (the PESQ front end shifts tiles whose peak lies outside
 *        [2^-40, 2^40] by a power of two; measured at common scales 1e-15 and 1e18: within
 *        5.6e-5 of the reference in every row) and DC offsets (the pre-emphasis runs FIR first,
 *        as the reference; +100 / +1000 on both signals: within 2.1e-3 in every row).
 *      STOI/ESTOI: scale-invariant from about 1e-10 to 1e17; below, the reference's own
 *        result is its 1e-12 * randn term (two seeds differ by 1e-2 around 0) and the engine
 *        returns that term's expectation (0; within 3.5e-3 of the reference in every row);
 *        above, float32 |X|^2 overflows and both give NaN.  DC offsets up to 1000x the signal:
 *        within 9.7e-3 in every row (the reference's own re-evaluations of those rows -- the
 *        same input scaled by 0.6 ... 1.3, another seed -- spread by up to 2.3e-2); a denoised
 *        signal 80-100 dB below the clean one in its upper bands: within 2.5e-4.  Pure tones
 *        (envelopes flat to ~1e-6, scores near 0): within 6.1e-3 (STOI) / 1.6e-2 (ESTOI) of the
 *        reference in every row, each inside twice that row's own re-evaluation spread
 *        (1.1e-2 / 2.1e-2 on the worst row);
 *  - return 0 on success or a negative FSEM_E* code (fsem_strerror() for text);
 *  - re-entrant across streams / devices (launches use the current HIP device).
 */
#ifndef FSEM_H
#define FSEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSEM_OK 0
#define FSEM_EINVAL -1        /* bad argument (sizes, null pointers)               */
#define FSEM_EWORKSPACE -2    /* workspace smaller than *_workspace_bytes()        */
#define FSEM_ELAUNCH -3       /* HIP launch / runtime error                        */
#define FSEM_ESHORT -4        /* input too short for the metric (see each entry)  */
#define FSEM_ERATE -5         /* unsupported sample-rate pair (see resampling)      */

const char *fsem_strerror(int code);
int fsem_version(void);  /* 10: + fsem_pesq_wb_frames_f32; 9: + fsem_pesq_bad_intervals_*, fsem_pesq_pool_f32; 8: + fsem_time_align_p862_*; 7: + fsem_host_buffer_mapped; 6: + fsem_build_id; 5: + fsem_time_align_utt_*; 4: + fsem_pre_emphasize_f32; 3: time alignment, distances */
/* Content hash (16 hex digits) of the sources, headers and compile flags this library was built
 * from (fast_speech_enhancement_metrics_amd/_build.py source_hash); the host layer refuses a
 * library whose id differs from its own tree's.  "unknown" for builds outside _build.py. */
const char *fsem_build_id(void);
/* 1 when the page-locked host buffer p is mapped into the device address space at the same
 * address (so an entry may write its scores straight into it), else 0.  Host-side query, no
 * kernel. */
int fsem_host_buffer_mapped(const void *p);

/* ---------------------------------------------------------------- resampling
 * torchaudio.transforms.Resample(orig, new) (sinc_interp_hann, width 6,
 * rolloff 0.99) as used by BaseMetric.prepare_audio   fast_se_metrics/base.py:13,19-20
 * out: [rows, fsem_resample_length(n_in, orig, new)] with row stride ld_out.
 * Any rate pair whose filter has at most 8192 taps (taps = 2 * ceil(6 * o / (0.99 * min(o, n))) + o
 * for the reduced pair o -> n = orig / g -> new / g): every common audio rate (8, 11.025, 16,
 * 22.05, 24, 32, 44.1, 48, 88.2, 96 kHz) to 16 or 10 kHz.  Longer filters (e.g. 44100 -> 16001)
 * give FSEM_ERATE here and in every entry that resamples (fsem_resample_length returns -1).
 * rows: any count (launches are sliced internally; no grid-dimension limit reaches the caller).
 */
int64_t fsem_resample_length(int64_t n_in, int32_t orig_freq, int32_t new_freq);
int fsem_resample_f32(const float *in, int64_t rows, int64_t n_in, int64_t ld_in,
                      float *out, int64_t ld_out, int32_t orig_freq, int32_t new_freq,
                      void *stream);
/* Ragged rows: row r is resampled as its first lengths[r] samples alone (zeros past them, as
 * BaseMetric.__call__'s zero-padded rows), giving fsem_resample_length(lengths[r], ...) samples;
 * the rest of the row, up to fsem_resample_length(n_in, ...), is written as zeros.
 * FSEM_ERATE if orig_freq == new_freq. */
int fsem_resample_rows_f32(const float *in, int64_t rows, int64_t n_in, int64_t ld_in,
                           const int32_t *lengths, float *out, int64_t ld_out, int32_t orig_freq,
                           int32_t new_freq, void *stream);

/* ---------------------------------------------------------------- PESQ-wb
 * Whole-metric entry: replaces PESQ.compute_metric    fast_se_metrics/PESQ.py:232-245
 * (get_disturbances :174-230 + MOS mapping :240-243) for 16 kHz input.
 *   ref, deg : [batch, length] float32 (row stride ld)  -- clean / denoised
 *   mos      : [batch] float32 output
 *   lengths  : NULL or [batch] int32 per-row lengths (see Conventions)
 * FSEM_ESHORT when the padded length yields < 20 frames (the reference's
 * unfold(1, 20, 10) raises RuntimeError there, PESQ.py:169); with `lengths`, such rows
 * give NaN.
 */
size_t fsem_pesq_workspace_bytes(int64_t batch, int64_t length);
int fsem_pesq_frames(int64_t length);  /* F = 1 + (L + L%256 - 512) / 256 (PESQ.py:128-133) */
int fsem_pesq_wb_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                     int64_t ld, const int32_t *lengths, float *mos, void *ws, size_t ws_bytes,
                     void *stream);

/* Stage entries (same math, split for parity tests of intermediates):
 * front: replaces PESQ.align_level's filtered power (PESQ.py:92-98) and
 *        PESQ.get_bark_bands (PESQ.py:123-140) up to BarkFilterBank.forward
 *        (bark.py:203-204), BEFORE the level scale:
 *          bark  [2*batch, 49, Fld] float32, band-major (signal s, band k, frame f at
 *                (s*49 + k)*Fld + f; signals 0..B-1 ref, B..2B-1 deg), unscaled,
 *                F = fsem_pesq_frames(length), Fld = F rounded up to a multiple of 32
 *                (frames F..Fld-1 unused); a shorter row fills its first
 *                fsem_pesq_frames(lengths[b]) frames
 *          power [2*batch] float32 = sum_t filtered^2 (not yet / (L+5120) / 1.04684)
 * back:  replaces PESQ.py:142-245 on those tensors -> mos [batch].
 */
size_t fsem_pesq_front_workspace_bytes(int64_t batch, int64_t length);
int fsem_pesq_front_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                        int64_t ld, const int32_t *lengths, float *bark, float *power, void *ws,
                        size_t ws_bytes, void *stream);
/* front_y10: the joint entry's front end -- as front, and also writes the rows' 10 kHz
 *        resampled signals (STOI's BaseMetric resampler, base.py:19-20) from the same tiles:
 *          y10 [2*batch, y_ld] float32, row 2b = clean b, 2b+1 = denoised b, first
 *          ceil(5*length_b/8) samples written; y_ld >= ceil(5*length/8), y_ld % 4 == 0;
 *          vad NULL or [batch, vad_ld, 2] float32: the clean rows' STOI voice-activity
 *          quarter sums (remove_silent_frames' frame energies, STOI.py:92-99, per 64-sample
 *          block m: {sum (w[64(m&1)+t] y[64m+t])^2, sum (w[128+64(m&1)+t] y[64m+t])^2}, w =
 *          hann(257)[1:]) for every complete block; vad_ld >= floor(L10/64)+1 rounded up to 64.
 */
int fsem_pesq_front_y10_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                            int64_t ld, const int32_t *lengths, float *bark, float *power,
                            float *y10, int64_t y_ld, float *vad, int64_t vad_ld, void *ws,
                            size_t ws_bytes, void *stream);
size_t fsem_pesq_back_workspace_bytes(int64_t batch, int64_t length);
int fsem_pesq_back_f32(const float *bark, const float *power, int64_t batch, int64_t length,
                       const int32_t *lengths, float *mos, void *ws, size_t ws_bytes,
                       void *stream);
/* distances: the back end's intermediates instead of the scores -- replaces
 *        PESQ.get_disturbances (PESQ.py:174-230) on the front end's tensors:
 *          dist   [2, batch] float32: symmetric distance (row 0) and asymmetric distance (row 1)
 *                 after get_overlapping_sums (PESQ.py:227-228); NaN for rows under 20 frames
 *          frames NULL or [batch, 2, Fcap] float32 (Fcap = fsem_pesq_frames(length)): per-frame
 *                 symmetric / asymmetric disturbances after the frame weighting and the clamp at
 *                 45 (PESQ.py:222-224); row b fills its first fsem_pesq_frames(lengths[b]) frames
 */
/* pre-emphasis: replaces the lfilter of PESQ.pre_emphasize (PESQ.py:111; the edge taper of
 *        :108-109 is the caller's, applied in place as the reference does) on any [rows, length]
 *        float32 rows: y = lfilter(x, a = (1, -1.9444777, 0.94597794), b = (2.740826,
 *        -5.4816519, 2.740826)) in torchaudio's float32 evaluation order (FIR then the all-pole
 *        loop).  y [rows, length] float32, row stride ld_out (y may equal x only if ld_out == ld).
 */
int fsem_pre_emphasize_f32(const float *x, int64_t rows, int64_t length, int64_t ld, float *y,
                           int64_t ld_out, void *stream);
size_t fsem_pesq_distances_workspace_bytes(int64_t batch, int64_t length);
int fsem_pesq_distances_f32(const float *bark, const float *power, int64_t batch, int64_t length,
                            const int32_t *lengths, float *dist, float *frames, void *ws,
                            size_t ws_bytes, void *stream);
/* wb_frames (ABI 10): fsem_pesq_wb_f32 with the distances and per-frame disturbances of
 *        fsem_pesq_distances_f32 beside the scores (dist [2, batch], frames [batch, 2, Fcap] as
 *        there), from the rows as given: the whole-metric path's range handling, where the
 *        stage entries need rows of moderate range.  Workspace: fsem_pesq_workspace_bytes.
 *        Used by the P.862 mode's bad-interval realignment (fsem_pesq_bad_intervals_f32).
 */
int fsem_pesq_wb_frames_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                            int64_t ld, const int32_t *lengths, float *mos, float *dist, float *frames,
                            void *ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------- STOI / ESTOI
 * Whole-metric entry: replaces STOI.compute_stoi + compute_metric
 *   fast_se_metrics/STOI.py:153-205 (after BaseMetric resampling to 10 kHz,
 *   base.py:19-20, when sample_rate != 10000).
 *   ref, deg    : [batch, length] float32 at `sample_rate` (row stride ld)
 *   lengths     : NULL or [batch] int32 per-row lengths at `sample_rate` (Conventions)
 *   stoi, estoi : [batch] float32 outputs; NaN where no 30-frame segment exists
 *                 (the reference warns there, STOI.py:163-165).
 */
size_t fsem_stoi_workspace_bytes(int64_t batch, int64_t length, int32_t sample_rate);
int fsem_stoi_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                  int64_t ld, const int32_t *lengths, int32_t sample_rate, float *stoi,
                  float *estoi, void *ws, size_t ws_bytes, void *stream);

/* Intermediates of the 10 kHz STOI pipeline for parity tests:
 *   kept  [batch] int32   -- frames kept by remove_silent_frames (STOI.py:88-111)
 *   tob   [2*batch, 15, tmax] float32 third-octave band envelopes (STOI.py:121-125),
 *         rows 0..B-1 ref, B..2B-1 deg; frames >= kept-2 are left untouched.
 * Input must already be at 10 kHz (length = 10 kHz samples).
 */
int fsem_stoi_tob_f32(const float *ref10, const float *deg10, int64_t batch,
                      int64_t length10, int64_t ld, int32_t *kept, float *tob, int64_t tmax,
                      void *ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------- joint PESQ + STOI
 * Both metrics of 16 kHz pairs from ONE read of the inputs: replaces the
 * reference's two calls PESQ(16000).compute_metric (PESQ.py:232-245) and
 * STOI(16000)(...) (base.py:19-20 resampling + STOI.py:153-205).  The PESQ front end's LDS
 * tiles also feed the fused 16 -> 10 kHz resampler.  Scores are bitwise those of
 * fsem_pesq_wb_f32 and fsem_stoi_f32(sample_rate = 16000) on the same rows.
 *   lengths : NULL or [batch] int32 per-row lengths (Conventions)
 *   mos, stoi, estoi : [batch] float32 outputs
 * FSEM_ESHORT (whole-batch form) when either metric's minimum length is not met.
 */
size_t fsem_pesq_stoi_workspace_bytes(int64_t batch, int64_t length);
int fsem_pesq_stoi_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                       int64_t ld, const int32_t *lengths, float *mos, float *stoi, float *estoi,
                       void *ws, size_t ws_bytes, void *stream);

/* ---------------------------------------------------------------- time alignment (opt-in)
 * NOT in the reference, whose PESQ has no time alignment (fast_se_metrics/PESQ.py:19-22); the
 * PESQ(..., time_align=True) extension calls this before the PESQ entries.
 * Per row pair of 16 kHz signals, after ITU-T P.862 section 10 (restated in
 * oracle/align_oracle.py; parity against P.862 implementations unpinned):
 *   crude delay from 4 ms voice-activity log envelopes (|delay| <= max_delay samples, rounded
 *   up to 4 ms frames), then the sample lag within +-383 of it maximising the cross-correlation
 *   of the signals' first differences.  delay[b] = D > 0: deg lags ref, deg[n] ~ ref[n - D].
 *   ref, deg    : [batch, length] float32 (row stride ld, ld % 4 == 0, 16-byte aligned rows)
 *   lengths     : NULL or [batch] int32 per-row lengths (Conventions)
 *   delay       : NULL or [batch] int32 output (at least one of delay / deg_aligned)
 *   deg_aligned : NULL or [batch, length] float32 output (row stride ld_out, ld_out % 4 == 0,
 *                 16-byte aligned rows):
 *                 deg_aligned[b][n] = deg[b][n + D] where 0 <= n + D < lengths[b], else 0
 *                 (not in place: deg_aligned must not overlap deg)
 * Cost: dominated by the fine search (fast correlation per 1280-sample block); see csrc/align.hip.
 */
size_t fsem_time_align_workspace_bytes(int64_t batch, int64_t length);
int fsem_time_align_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                        int64_t ld, const int32_t *lengths, int32_t max_delay, int32_t *delay,
                        float *deg_aligned, int64_t ld_out, void *ws, size_t ws_bytes,
                        void *stream);

/* utterance mode (ABI 5): P.862's per-utterance alignment (sections 10.3-10.5, restated in
 * oracle/align_oracle.py steps 5-9; parity against P.862 implementations unpinned):
 *   utterances of the reference (envelope speech runs of 16 ms or more, joined across gaps < 200 ms, at
 *   least 200 ms, at most 16 per row) each own a region of the row (boundaries in the middle of
 *   the gaps); per utterance a crude delay (envelope correlation over the utterance +-300 ms,
 *   within +-300 ms of the row's crude delay), then the fine delay of its region as above; a
 *   region splits once at a 5120-sample piece boundary when two delays (>= 16 samples apart)
 *   raise the summed correlation peak by 20 %.  Consecutive segments of equal delay are merged.
 *   delay     : NULL or [batch] int32: the row's longest segment's delay (first of equals)
 *   n_seg     : NULL or [batch] int32 segment counts (1 .. FSEM_ALIGN_MAX_SEGMENTS)
 *   seg_start : NULL or [batch, FSEM_ALIGN_MAX_SEGMENTS + 1] int32: segment k of row b covers
 *               samples [seg_start[b][k], seg_start[b][k + 1]); seg_start[b][n_seg[b]] = lengths[b]
 *   seg_delay : NULL or [batch, FSEM_ALIGN_MAX_SEGMENTS] int32 delays (n_seg, seg_start and
 *               seg_delay: all three or none; at least one of delay / n_seg / deg_aligned)
 *   deg_aligned[b][n] = deg[b][n + D_k] for n in segment k where 0 <= n + D_k < lengths[b], else 0
 * Other arguments as fsem_time_align_f32.
 */
#define FSEM_ALIGN_MAX_SEGMENTS 32
size_t fsem_time_align_utt_workspace_bytes(int64_t batch, int64_t length);
int fsem_time_align_utt_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                            int64_t ld, const int32_t *lengths, int32_t max_delay, int32_t *delay,
                            int32_t *n_seg, int32_t *seg_start, int32_t *seg_delay,
                            float *deg_aligned, int64_t ld_out, void *ws, size_t ws_bytes,
                            void *stream);

/* P.862 mode (ABI 8): the utterance mode's stages up to the per-piece correlations, then P.862's
 * histogram fine alignment and recursive utterance split (sections 10.5-10.6, restated in
 * oracle/align_oracle.py steps 10-12 on the 5120-sample pieces instead of P.862's 64 ms frames;
 * parity against P.862 implementations unpinned): every piece whose correlation peak reaches
 * 5 % of its utterance's largest votes for its peak lag with weight peak^0.125; a range of
 * pieces takes the first maximum of its triangle-smoothed (+-8 lags) vote histogram as delay and
 * that maximum's share of the votes as confidence; a range splits at the piece boundary whose two
 * halves (two or more votes each, delays >= 16 samples apart) are both more confident than the
 * whole, the largest summed confidence first, and each half is tried once more (up to 4 segments
 * per utterance; at most FSEM_ALIGN_MAX_SEGMENTS per row, later ones merging into the last).
 * Arguments, outputs and workspace rules as fsem_time_align_utt_f32.  Replaces nothing in the
 * reference (its PESQ has no time alignment, fast_se_metrics/PESQ.py:19-22).
 */
size_t fsem_time_align_p862_workspace_bytes(int64_t batch, int64_t length);
int fsem_time_align_p862_f32(const float *ref, const float *deg, int64_t batch, int64_t length,
                             int64_t ld, const int32_t *lengths, int32_t max_delay, int32_t *delay,
                             int32_t *n_seg, int32_t *seg_start, int32_t *seg_delay,
                             float *deg_aligned, int64_t ld_out, void *ws, size_t ws_bytes,
                             void *stream);

/* bad intervals (ABI 9): P.862's realignment of bad intervals after the perceptual model (section
 * 10.7, restated in oracle/align_oracle.py steps 13-15; parity against P.862 implementations
 * unpinned), for the P.862 mode's rows.  Replaces nothing in the reference.
 *   deg_aligned : [batch, length] float32 (row stride ld_out): fsem_time_align_p862_f32's output
 *   frames      : [batch, 2, Fcap] float32 (Fcap = fsem_pesq_frames(length)): the per-frame
 *                 disturbances of (ref, deg_aligned), fsem_pesq_wb_frames_f32's (or
 *                 fsem_pesq_distances_f32's)
 *   n_seg, seg_start, seg_delay : that alignment's segments
 *   n_bad       : [batch] int32 output: intervals per row (0 .. FSEM_PESQ_MAX_BAD)
 *   bad         : [batch, FSEM_PESQ_MAX_BAD, 3] int32 output: {first frame, end frame, delay} --
 *                 runs of frames with symmetric disturbance > 30, joined across gaps < 4 frames,
 *                 from 5 frames long, in order; delay: the first maximum of the first-difference
 *                 correlation over the interval's samples [256 f0, min(256 f1 + 256, lengths[b]))
 *                 within +-383 of the delay of the segment holding its first sample (that delay
 *                 when no lag correlates positively)
 *   deg_second  : [batch, length] float32 output (row stride ld_out; may be deg_aligned itself):
 *                 deg[b][n + delay_i] for n in interval i (0 <= n + delay_i < lengths[b], else 0),
 *                 deg_aligned[b][n] elsewhere
 * pool: the MOS of each row from the first frames, an interval taking frames2 (the per-frame
 *   disturbances of (ref, deg_second)) when their symmetric sum over it is smaller; the pooling
 *   and mapping of fsem_pesq_wb_f32 (PESQ.py:168-172, 240-243).  dist: [2, batch] the first
 *   distances (NaN there gives NaN); rows under 20 frames give NaN.
 */
#define FSEM_PESQ_MAX_BAD 16
size_t fsem_pesq_bad_intervals_workspace_bytes(int64_t batch, int64_t length);
int fsem_pesq_bad_intervals_f32(const float *ref, const float *deg, const float *deg_aligned, int64_t batch,
                                int64_t length, int64_t ld, const int32_t *lengths, const float *frames,
                                const int32_t *n_seg, const int32_t *seg_start, const int32_t *seg_delay,
                                int32_t *n_bad, int32_t *bad, float *deg_second, int64_t ld_out, void *ws,
                                size_t ws_bytes, void *stream);
int fsem_pesq_pool_f32(const float *frames, const float *frames2, const float *dist, int64_t batch,
                       int64_t length, const int32_t *lengths, const int32_t *n_bad, const int32_t *bad,
                       float *mos, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FSEM_H */

/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * CPU restatement of torchaudio 2.8.0's `torchaudio.functional.lfilter`
 * (third-party dependency of the reference, absent from /root/reference and
 * from this image).  The reference calls it at
 *   fast_se_metrics/PESQ.py:94   (10th-order Butterworth band-pass, clamp=False)
 *   fast_se_metrics/PESQ.py:111  (2nd-order pre-emphasis, clamp=False)
 *
 * torchaudio's published algorithm (functional/filtering.py `_lfilter` +
 * the CPU `_lfilter_core_cpu_loop`):
 *   1. FIR part: w[n] = sum_j b_flip[j] * xpad[n + j], xpad = x left-padded with
 *      (order-1) zeros, computed by conv1d, then divided by a[0];
 *   2. a_flip = flip(a) / a[0];
 *   3. sequential fp32 loop over n:
 *        acc = w[n];
 *        for i in 0..order-1: acc -= ypad[n + i] * a_flip[i];   (oldest first)
 *        ypad[n + order - 1] = acc;
 *      where ypad is the output left-padded with (order-1) zeros; the i = order-1
 *      term multiplies the not-yet-written (zero) slot.
 * Everything is float32, exactly the operation order above.  The FIR sum order
 * of conv1d is an implementation detail of oneDNN; we use j ascending.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* x, y: [rows, n] float32 row-major; a, b: [order] float32 (order = len). */
int oracle_lfilter_f32(const float *x, float *y, int64_t rows, int64_t n,
                       const float *a, const float *b, int order) {
    if (order <= 0 || order > 64) return -1;
    float a_flip[64], b_flip[64];
    const float a0 = a[0];
    for (int i = 0; i < order; ++i) {
        a_flip[i] = a[order - 1 - i] / a0;
        b_flip[i] = b[order - 1 - i];
    }
    const int64_t pad = order - 1;
    float *ypad = (float *)malloc(sizeof(float) * (size_t)(n + pad));
    if (!ypad) return -2;
    for (int64_t r = 0; r < rows; ++r) {
        const float *xr = x + r * n;
        memset(ypad, 0, sizeof(float) * (size_t)(n + pad));
        for (int64_t t = 0; t < n; ++t) {
            /* FIR (conv1d over the left-padded input), then / a0 */
            float w = 0.0f;
            for (int j = 0; j < order; ++j) {
                const int64_t src = t + j - pad;
                if (src >= 0) w += b_flip[j] * xr[src];
            }
            w = w / a0;
            float acc = w;
            for (int i = 0; i < order; ++i) acc -= ypad[t + i] * a_flip[i];
            ypad[t + pad] = acc;
        }
        memcpy(y + r * n, ypad + pad, sizeof(float) * (size_t)n);
    }
    free(ypad);
    return 0;
}

/* IIR part only, input already FIR-filtered (w), torchaudio loop order. */
int oracle_lfilter_iir_f32(const float *w, float *y, int64_t rows, int64_t n,
                           const float *a_flip_norm, int order) {
    if (order <= 0 || order > 64) return -1;
    const int64_t pad = order - 1;
    float *ypad = (float *)malloc(sizeof(float) * (size_t)(n + pad));
    if (!ypad) return -2;
    for (int64_t r = 0; r < rows; ++r) {
        memset(ypad, 0, sizeof(float) * (size_t)(n + pad));
        const float *wr = w + r * n;
        for (int64_t t = 0; t < n; ++t) {
            float acc = wr[t];
            for (int i = 0; i < order; ++i) acc -= ypad[t + i] * a_flip_norm[i];
            ypad[t + pad] = acc;
        }
        memcpy(y + r * n, ypad + pad, sizeof(float) * (size_t)n);
    }
    free(ypad);
    return 0;
}

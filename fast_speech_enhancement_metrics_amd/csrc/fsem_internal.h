// Internal (non-exported, C++) entry points shared between the engine's translation units;
// the joint PESQ + STOI entry (fsem_pesq_stoi_f32, stoi.hip) composes them.
#pragma once
#include "fsem_common.h"

namespace fsem {
// A side stream on `st`'s device (one per device, created on first use, lives with the process)
// for work that can overlap the caller's stream; `st` itself when none can be had.
hipStream_t side_stream(hipStream_t st);
// Make `waiter` wait for everything queued on `producer` so far (no-op when they are the same).
int stream_wait(hipStream_t waiter, hipStream_t producer);
// Compute units of the current device (queried once per device).
int cu_count();

namespace pesq {
// pesq_front + power sums; with y10 != nullptr also writes the rows' 10 kHz resampled signals
// ([2*batch, y_ld], row 2b = clean b, 2b+1 = denoised b) from the same LDS tiles, and with
// vad != nullptr the clean rows' STOI VAD quarter sums ([batch, v_ld] float2, fsem_vad.h).
// power_sums false: no per-signal power sums (the per-segment partials stay at the start of ws
// for launch_back)
int launch_front(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                 const int32_t *lengths, float *bark, float *power, void *ws, size_t ws_bytes, float *y10,
                 int64_t y_ld, float2 *vad, int64_t v_ld, hipStream_t st, bool power_sums = true);
// pesq_back over bark with the signal powers given (power) or summed from the front end's
// per-segment partials (ppart, power == nullptr); ws as fsem_pesq_back_workspace_bytes
int launch_back(const float *bark, const float *power, const float *ppart, int64_t batch, int64_t length,
                const int32_t *lengths, float *mos, void *ws, size_t ws_bytes, hipStream_t stream,
                float *dist = nullptr, float *frames = nullptr);
// the two halves of run_wb on one workspace (fsem_pesq_workspace_bytes): the front end (as
// launch_front) and, once it is complete on back_st, the back end writing mos
int run_wb_front(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld,
                 const int32_t *lengths, void *ws, size_t ws_bytes, float *y10, int64_t y_ld, float2 *vad,
                 int64_t v_ld, hipStream_t st);
int run_wb_back(int64_t batch, int64_t length, const int32_t *lengths, float *mos, void *ws, hipStream_t back_st);
// whole PESQ-wb (front + back), optionally emitting y10 as above; the back end runs on back_st
// after the front end on st (back_st == st: one stream)
int run_wb(const float *ref, const float *deg, int64_t batch, int64_t length, int64_t ld, const int32_t *lengths,
           float *mos, void *ws, size_t ws_bytes, float *y10, int64_t y_ld, float2 *vad, int64_t v_ld,
           hipStream_t st, hipStream_t back_st);
// waves per utterance of the back end for this batch (1, 4 or 8; pesq.hip) and the LDS the
// one-wave form needs for its keep ballots
int back_waves(int64_t batch, int64_t length);
size_t back_keep_bytes(int64_t length);
}  // namespace pesq
}  // namespace fsem

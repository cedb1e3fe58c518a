// PESQ-wb back end for gfx950 (MI355X): level scale, silent frames, band and frame
// equalisation, Zwicker loudness, disturbances, L6/L2 pooling and the MOS mapping
// (fast_se_metrics/PESQ.py:142-245, utils/loudness.py:48-67, utils/bark.py:169-184) over the
// front end's Bark bands (pesq.hip).  Its own translation unit: compiled WITH the SLP
// vectoriser (its 49-band loops pack into v_pk_* pairs), the front end without
// (_build.SOURCE_FLAGS).
#include "fsem_fft.h"  // (the constant tables, fsem_tables.inc)
#include "fsem_internal.h"
#include "fsem_pesq.h"

namespace fsem {
namespace pesq {

// ------------------------------------------------------------------------------ back end
// x^e for x > 0 (every call site: x >= 0.5 or a ratio of positive terms) via the hardware
// v_log_f32 / v_exp_f32 (~1 ulp each); the reference evaluates these in float64, the
// difference is ~1e-7 relative, far inside the +-0.01 MOS tolerance.
__device__ __forceinline__ float pow_pos(float x, float e) {
  return __builtin_amdgcn_exp2f(e * __builtin_amdgcn_logf(x));
}

__device__ __forceinline__ float loud(float p, int b) {
  // loudness.py:64-65: (2T)^e ((0.5 + 0.5 P/T)^e - 1), 0 where P <= T; times Sl (folded).
  // 0.5 P/T as P * (0.5/T) (one rounding instead of a correctly rounded division: <=1 ulp)
  // branch-free (p >= 0: the pow argument is >= 0.5 either way)
  const float v = kLoud2TE[b] * (pow_pos(fmaf(p, kHalfInvThresh[b], 0.5f), kLoudExp[b]) - 1.f);
  return (p > kThresh[b]) ? v : 0.f;
}

// BW waves per utterance, lane = frame: each load brings one band of 64 consecutive frames
// (band-major rows, bark_ld), straight into registers -- no LDS staging, so occupancy is set
// by VGPRs alone (the frame's 49 clean and 49 denoised band values stay in registers per chunk).
// The utterance's chunks are dealt round-robin to its waves.  BW = 1 for batches that fill the
// chip (no barriers, no idle waves at the end of an utterance: the throughput form); BW = 4 for
// small batches, where one utterance's latency is the call's.  The two differ only in the
// summation order of the band totals and of the window L2 sum (~1e-7 relative in the score).
// STAGE: the stage entry's instance (fsem_pesq_distances_f32), which also writes the distances
// and the per-frame disturbances; the scoring instances carry no trace of those outputs.
template <int BW, bool STAGE = false>
__global__ void __launch_bounds__(64 * BW) __attribute__((amdgpu_waves_per_eu(4)))
    pesq_back(const float *__restrict__ bark, const float *__restrict__ power, const float *__restrict__ ppart,
              const int *__restrict__ pexp, int nseg, int64_t B, int64_t Lcap, const int32_t *__restrict__ lens, int Fcap,
              float *__restrict__ scratch, float *__restrict__ mos, float *__restrict__ dist,
              float *__restrict__ frames) {
  constexpr int BT = 64 * BW;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t b = blockIdx.x;
  const int64_t L = row_length(lens, b, Lcap);
  const int F = frames_of(L);  // this utterance's frames; rows are laid out with stride bark_ld(Fcap)
  if (F < 20) {  // the reference's unfold(1, 20, 10) raises here (PESQ.py:169)
    if (tid == 0) {
      mos[b] = __builtin_nanf("");
      if (STAGE && dist) dist[b] = dist[B + b] = __builtin_nanf("");
    }
    return;
  }
  const int64_t fld = bark_ld(Fcap);
  const float *__restrict__ bc = bark + b * NBARK * fld;
  const float *__restrict__ bn = bark + (b + B) * NBARK * fld;
  // band rows by raw buffer loads (voffset = 4 * (k * fld + frame))
  auto rsrc = [](const float *p, int64_t n) {
    const uint64_t base = reinterpret_cast<uint64_t>(p);
    // uint32_t: readfirstlane returns int, which would sign-extend into the high word
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    void *q = reinterpret_cast<void *>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, (int)(n * 4), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rcl = rsrc(bc, NBARK * fld), rdn = rsrc(bn, NBARK * fld);
  const int fstride = 4 * (int)fld;  // one signal's bands span < 2^29 floats
  auto ld = [](__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  };
  // scratch row of this utterance (stride 4 * Fcap): sym [0, F), asym [F, 2F), and with several
  // waves the keep flags from 2 Fcap on (one word per frame, written and read back by one lane)
  float *__restrict__ sym = scratch + b * (int64_t)Fcap * 4;
  float *__restrict__ asym = sym + F;
  int *__restrict__ keepf = reinterpret_cast<int *>(sym + 2 * (int64_t)Fcap);
  // PESQ.py:97-100 -- power = sum / (L + 5120) / 1.04684; bark scales by 1e7 / power
  // signal powers: given, or (ppart != nullptr, the whole-metric entries) summed here from the
  // front end's per-segment partials in pesq_power_sum's order -- one launch fewer per call
  // With range-shifted segments (pesq_front's pexp), the partials are summed at the largest
  // segment scale E (each scaled by 2^(-2 sh - E) <= 1) and frame f's bands by
  // 2^(-2 sh(f) - E) on top of the level scale; with every shift 0 (every input whose tile
  // peaks lie in [2^-40, 2^40]) the arithmetic is exactly the unshifted one.
  float pwc, pwn;
  int eC = 0, eN = 0;             // E of clean / denoised
  bool shc = false, shn = false;  // any segment shifted
  if (ppart) {
    __shared__ float pw_s[2];
    __shared__ int pe_s[2], ps_s[2];
    if (tid < 2) {
      const float *__restrict__ q = ppart + (b + tid * B) * (int64_t)nseg * 4;
      const int *__restrict__ ex = pexp + (b + tid * B) * (int64_t)nseg;
      int emax = -(1 << 30), any = 0;
      for (int g = 0; g < nseg; ++g) {
        emax = max(emax, -2 * ex[g]);
        any |= ex[g];
      }
      float acc = 0.f;
      for (int g = 0; g < 4 * nseg; ++g) acc += __builtin_amdgcn_ldexpf(q[g], -2 * ex[g >> 2] - emax);
      pw_s[tid] = acc;
      pe_s[tid] = emax;
      ps_s[tid] = any != 0;
    }
    lds_barrier();
    pwc = pw_s[0];
    pwn = pw_s[1];
    eC = pe_s[0];
    eN = pe_s[1];
    shc = ps_s[0] != 0;
    shn = ps_s[1] != 0;
  } else {
    pwc = power[b];
    pwn = power[b + B];
  }
  const float pc = pwc / (float)(L + 5120) / 1.04684f;
  const float pn = pwn / (float)(L + 5120) / 1.04684f;
  const float sc = 1e7f / pc, sn = 1e7f / pn;
  const int *__restrict__ exc = pexp ? pexp + b * (int64_t)nseg : nullptr;
  const int *__restrict__ exn = pexp ? pexp + (b + B) * (int64_t)nseg : nullptr;
  // the level scale of frame f (per lane: frames of one chunk may lie in two segments)
  auto scale_at = [&](bool shifted, const int *__restrict__ ex, int E, float s0, int f) {
    return shifted ? __builtin_amdgcn_ldexpf(s0, -2 * ex[f / NF] - E) : s0;
  };
  const int nch = (F + 63) / 64;

  // ---- pass 1: silent frames (PESQ.py:146, loudness.py:48-53 x 1e2) and per-lane partial band
  // sums of the audible power of non-silent frames (loudness.py:55-60).  The clean sweep keeps
  // each frame's keep flag, so the denoised sums follow in a second sweep without the clean
  // accumulators live: one wave keeps a ballot per chunk in LDS ([ceil(Fcap / 64)], dynamic);
  // several waves keep a word per frame in the scratch row, each lane reading back its own.
  extern __shared__ unsigned long long keepm[];
  __shared__ float ratio_s[NBARK];
  __shared__ float red[BW][16 * 65];
  __shared__ float tot[2][BW][NBARK];
  __shared__ double dred[2][BW];
  float acc[NBARK];
#pragma unroll
  for (int k = 0; k < NBARK; ++k) acc[k] = 0.f;
  for (int c = wv; c < nch; c += BW) {
    const int f = 64 * c + lane;
    const bool valid = f < F;
    const int fi = valid ? f : F - 1;  // clamped: every load in bounds, results masked
    int fs = fstride;
    asm volatile("" : "+s"(fs));  // per-chunk: keeps the 49 band offsets out of live SGPRs
    float aud[NBARK];  // audible clean power of each band (values, not compare masks: SGPRs)
    float a = 0.f;
    const float scf = scale_at(shc, exc, eC, sc, fi);
#pragma unroll
    for (int k = 0; k < NBARK; ++k) {
      const float cl = ld(rcl, 4 * fi + k * fs, 0) * scf;
      aud[k] = (cl > kThresh[k] * 100.f) ? cl : 0.f;
      a += aud[k];
    }
    const bool keep = valid && !(a < 1e7f);
    if (BW == 1) {
      const unsigned long long km = __ballot(keep);
      if (lane == 0) keepm[c] = km;
    } else if (valid) {
      keepf[f] = keep;
    }
#pragma unroll
    for (int k = 0; k < NBARK; ++k) acc[k] += keep ? aud[k] : 0.f;
  }
  // lane-partial band sums -> this wave's totals by an LDS transpose, 16 bands per round (row =
  // band over the 64 lanes, stride 65: conflict-free both ways); lane k < 49 ends up holding
  // band k's total over the wave's chunks, which goes to tot[s][wave][k]
  auto band_totals = [&](float v[NBARK], int s) {
    float t = 0.f;
    float *rw = red[wv];
#pragma unroll
    for (int k0 = 0; k0 < NBARK; k0 += 16) {
#pragma unroll
      for (int k = k0; k < k0 + 16 && k < NBARK; ++k) rw[(k - k0) * 65 + lane] = v[k];
      wave_lds_fence();
      if (lane >= k0 && lane < k0 + 16 && lane < NBARK) {
#pragma unroll 16
        for (int j = 0; j < 64; ++j) t += rw[(lane - k0) * 65 + j];
      }
      wave_lds_fence();
    }
    if (lane < NBARK) tot[s][wv][lane] = t;
  };
  band_totals(acc, 0);
  if (BW > 1) __threadfence_block();  // the keep flags, read back below
#pragma unroll
  for (int k = 0; k < NBARK; ++k) acc[k] = 0.f;
  for (int c = wv; c < nch; c += BW) {
    const int f = 64 * c + lane;
    const int fi = f < F ? f : F - 1;
    int fs = fstride;
    asm volatile("" : "+s"(fs));
    const bool keep = (BW == 1) ? ((keepm[c] >> lane) & 1ull) : ((f < F) && keepf[fi]);
    const float snf = scale_at(shn, exn, eN, sn, fi);
#pragma unroll
    for (int k = 0; k < NBARK; ++k) {
      const float n = ld(rdn, 4 * fi + k * fs, 0) * snf;
      acc[k] += (keep && n > kThresh[k] * 100.f) ? n : 0.f;
    }
  }
  band_totals(acc, 1);
  lds_barrier();
  // band power ratio (PESQ.py:151-152), wave totals summed in wave order
  if (tid < NBARK) {
    float mc = 0.f, mn = 0.f;
#pragma unroll
    for (int w = 0; w < BW; ++w) {
      mc += tot[0][w][tid];
      mn += tot[1][w][tid];
    }
    const float cm = mc / (float)F, nm = mn / (float)F;
    ratio_s[tid] = fminf(fmaxf((nm + 1000.f) / (cm + 1000.f), 0.01f), 100.f);
  }
  lds_barrier();

  // ---- pass 2: frame ratio (PESQ.py:157-163), loudness, disturbances (PESQ.py:186-224).
  // The ratio smoothing reads the previous frame's ratio: one wave carries it from chunk to
  // chunk; with several waves a chunk is 63 new frames plus, in lane 0, the frame before them
  // (its ratio only), so the chunks are independent.
  constexpr int CW = BW == 1 ? 64 : 63, OFF = BW == 1 ? 0 : 1;
  const float sqrt_tw = sqrtf((float)kTotalWidth);
  const int nch2 = (F + CW - 1) / CW;
  float fr_prev = 0.f;  // BW == 1: ratio of the previous chunk's last frame
  for (int c = wv; c < nch2; c += BW) {
    const int f = CW * c - OFF + lane;
    const bool valid = (OFF == 0 || lane > 0) && f < F;
    const int fi = f < 0 ? 0 : (f < F ? f : F - 1);
    int fs = fstride;
    asm volatile("" : "+s"(fs));
    float ec[NBARK], ns[NBARK];
    float ac = 0.f, an = 0.f;
    const float scf = scale_at(shc, exc, eC, sc, fi), snf = scale_at(shn, exn, eN, sn, fi);
#pragma unroll
    for (int k = 0; k < NBARK; ++k) {
      ec[k] = ratio_s[k] * (ld(rcl, 4 * fi + k * fs, 0) * scf);
      ns[k] = ld(rdn, 4 * fi + k * fs, 0) * snf;
      ac += (ec[k] > kThresh[k]) ? ec[k] : 0.f;
      an += (ns[k] > kThresh[k]) ? ns[k] : 0.f;
    }
    const float fr = (ac + 5e3f) / (an + 5e3f);
    float prev = __shfl_up(fr, 1, 64);
    if (OFF == 0) {
      if (lane == 0) prev = fr_prev;
      fr_prev = __shfl(fr, 63, 64);
    }
    float r = (f >= 1) ? 0.8f * fr + 0.2f * prev : fr;  // non-recursive (PESQ.py:161)
    r = fminf(fmaxf(r, 3e-4f), 5.f);
    float s2 = 0.f, as = 0.f;
#pragma unroll
    for (int k = 0; k < NBARK; ++k) {
      const float en = r * ns[k];
      const float lc = loud(ec[k], k), ln = loud(en, k);
      float d = ln - lc;
      const float dz = 0.25f * fminf(lc, ln);
      d = copysignf(fmaxf(fabsf(d) - dz, 0.f), d);
      if (k >= 1) {
        const float wd = kWidthBark[k] * d;
        s2 = fmaf(wd, wd, s2);
        float am = pow_pos((en + 50.f) * __builtin_amdgcn_rcpf(ec[k] + 50.f), 1.2f);  // ~1 ulp rcp
        am = (am < 3.f) ? 0.f : fminf(am, 12.f);
        as += fabsf(wd * am);
      }
    }
    const float sy = fmaxf(sqrt_tw * sqrtf(s2), 1e-20f);
    const float ay = fmaxf(as, 1e-20f);
    const float w = pow_pos((ac + 1e5f) / 1e7f, 0.04f);
    if (valid) {
      const float fs_ = fminf(sy / w, 45.f), fa_ = fminf(ay / w, 45.f);
      sym[f] = fs_;
      asym[f] = fa_;
      if (STAGE && frames) {  // stage entry only (fsem_pesq_distances_f32): [B, 2, Fcap]
        frames[(2 * b) * (int64_t)Fcap + f] = fs_;
        frames[(2 * b + 1) * (int64_t)Fcap + f] = fa_;
      }
    }
  }
  __syncthreads();  // pass 3 reads other waves' sym / asym stores
  // ---- pass 3: L6 within 20-frame windows (hop 10), L2 across windows (PESQ.py:168-172)
  const int nw = (F - 20) / 10 + 1;
  double as_ = 0.0, aa_ = 0.0;
  for (int w = tid; w < nw; w += BT) {
    double s6 = 0.0, a6 = 0.0;
    for (int i = 0; i < 20; ++i) {
      const double x = sym[10 * w + i], y = asym[10 * w + i];
      const double x2 = x * x, y2 = y * y;
      s6 += x2 * x2 * x2;
      a6 += y2 * y2 * y2;
    }
    const double ps = pow(s6 / 20.0, 1.0 / 6.0), pa = pow(a6 / 20.0, 1.0 / 6.0);
    as_ += ps * ps;
    aa_ += pa * pa;
  }
  as_ = wave_sum_d(as_);
  aa_ = wave_sum_d(aa_);
  if (lane == 0) {
    dred[0][wv] = as_;
    dred[1][wv] = aa_;
  }
  lds_barrier();
  if (tid == 0) {
    double ts = 0.0, ta = 0.0;
#pragma unroll
    for (int w = 0; w < BW; ++w) {
      ts += dred[0][w];
      ta += dred[1][w];
    }
    const double ds = sqrt(ts / nw), da = sqrt(ta / nw);
    double m = 4.5 - 0.1 * ds - 0.0309 * da;              // PESQ.py:240
    m = 0.999 + 4.0 / (1.0 + exp(-1.3669 * m + 3.8224));  // PESQ.py:243
    // a signal with zero (or non-finite) band-pass power: the reference's x * sqrt(1e7 / power)
    // (PESQ.py:100) turns it into NaN samples, which torch's clamp / pow propagate to the score;
    // here the scale multiplies Bark bands whose NaNs the comparisons above would drop
    const bool fin = __builtin_isfinite(sc) && __builtin_isfinite(sn);
    mos[b] = fin ? (float)m : __builtin_nanf("");
    if (STAGE && dist) {  // stage entry only: the symmetric / asymmetric distances (PESQ.py:227-230)
      dist[b] = fin ? (float)ds : __builtin_nanf("");
      dist[B + b] = fin ? (float)da : __builtin_nanf("");
    }
  }
}

}  // namespace pesq
}  // namespace fsem

using namespace fsem;

size_t fsem::pesq::back_keep_bytes(int64_t length) {
  return sizeof(unsigned long long) * (size_t)((pesq::geometry(length).F + 63) / 64);
}

// Waves per utterance of the back end: several for small batches, where one utterance's latency
// is the call's (10 s rows, B = 256: 4 waves 0.083 ms vs one 0.100 ms; 16 s rows, B = 64: PESQ
// call 0.268 ms with 4 waves, 0.232 ms with 8, which a joint call at B = 256 loses back by
// crowding the STOI kernels beside it: 8 up to half a row per CU, then 4); one wave once the batch
// gives every CU more than 2 rows (from B = 1024 one wave is as fast or faster, and leaves more
// room to the STOI segment kernel beside it in the joint entry); one wave also needs its keep
// ballots in LDS.  FSEM_BACK_WAVES (diagnostics only) forces 1, 4 or 8.
int fsem::pesq::back_waves(int64_t batch, int64_t length) {
  static const int forced = [] {
    const char *e = getenv("FSEM_BACK_WAVES");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 4 || v == 8) ? v : 0;
  }();
  const bool fits = back_keep_bytes(length) <= 32768;
  if (forced) return (forced == 1 && !fits) ? 4 : forced;
  const int ncu = cu_count();
  if (fits && batch > 2 * (int64_t)ncu) return 1;
  return batch > ncu / 2 ? 4 : 8;
}

extern "C" size_t fsem_pesq_back_workspace_bytes(int64_t batch, int64_t length) {
  const pesq::Geometry g = pesq::geometry(length);
  return align_up(sizeof(float) * (size_t)batch * (size_t)g.F * 4, 256);
}

int fsem::pesq::launch_back(const float *bark, const float *power, const float *ppart, int64_t batch,
                            int64_t length, const int32_t *lengths, float *mos, void *ws, size_t ws_bytes,
                            hipStream_t stream, float *dist, float *frames) {
  if (!bark || (!power && !ppart) || !mos || batch <= 0 || length <= 0 || length > kMaxLength) return FSEM_EINVAL;
  const pesq::Geometry g = pesq::geometry(length);
  if (g.F < 20 && !lengths) return FSEM_ESHORT;
  if (!ws || ws_bytes < fsem_pesq_back_workspace_bytes(batch, length)) return FSEM_EWORKSPACE;
  if (batch > 0x7fffffff) return FSEM_EINVAL;
  const int bw = pesq::back_waves(batch, length);
  float *scratch = static_cast<float *>(ws);
  // with the front end's partials, its range shifts follow them (fsem_pesq_front_workspace_bytes)
  const int *pexp = ppart ? reinterpret_cast<const int *>(reinterpret_cast<const char *>(ppart) +
                                                          pesq::front_ppart_bytes(batch, length))
                          : nullptr;
#define FSEM_BACK(W, S, LDS)                                                                                   \
  hipLaunchKernelGGL((pesq::pesq_back<W, S>), dim3((unsigned)batch), dim3(64 * W), LDS, stream, bark, power, ppart, \
                     pexp, g.nseg, batch, length, lengths, g.F, scratch, mos, dist, frames)
  if (dist || frames) {
    if (bw == 8) FSEM_BACK(8, true, 0);
    else if (bw == 4) FSEM_BACK(4, true, 0);
    else FSEM_BACK(1, true, pesq::back_keep_bytes(length));
  } else {
    if (bw == 8) FSEM_BACK(8, false, 0);
    else if (bw == 4) FSEM_BACK(4, false, 0);
    else FSEM_BACK(1, false, pesq::back_keep_bytes(length));
  }
#undef FSEM_BACK
  FSEM_CHECK_LAUNCH();
  return FSEM_OK;
}

extern "C" int fsem_pesq_back_f32(const float *bark, const float *power, int64_t batch, int64_t length,
                                  const int32_t *lengths, float *mos, void *ws, size_t ws_bytes,
                                  void *stream) {
  if (!power) return FSEM_EINVAL;
  return pesq::launch_back(bark, power, nullptr, batch, length, lengths, mos, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" size_t fsem_pesq_distances_workspace_bytes(int64_t batch, int64_t length) {
  // the back end's scratch rows, then the scores it also writes
  return fsem_pesq_back_workspace_bytes(batch, length) + align_up(sizeof(float) * (size_t)batch, 256);
}

extern "C" int fsem_pesq_distances_f32(const float *bark, const float *power, int64_t batch, int64_t length,
                                       const int32_t *lengths, float *dist, float *frames, void *ws,
                                       size_t ws_bytes, void *stream) {
  if (!power || !dist || batch <= 0 || length <= 0) return FSEM_EINVAL;
  if (!ws || ws_bytes < fsem_pesq_distances_workspace_bytes(batch, length)) return FSEM_EWORKSPACE;
  const size_t back = fsem_pesq_back_workspace_bytes(batch, length);
  float *mos = reinterpret_cast<float *>(static_cast<char *>(ws) + back);
  return pesq::launch_back(bark, power, nullptr, batch, length, lengths, mos, ws, back, (hipStream_t)stream, dist,
                           frames);
}


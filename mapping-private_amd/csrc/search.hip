// search.hip -- sliding-box subspace search on gfx950.
//
// Replaces SearchObj{,Multi}::setData + searchPart (color_voxel_recognition/src/
// search.cpp:431-480, 539-658, 915-968).
//
// compress: G = f' * axis_p^T, an LDS-tiled fp32 GEMM (64 subdivisions x 128 dims per
//   workgroup, 4x8 register tile per thread, fma chain in ascending feature order);
//   setNormalizeVal's max-normalisation (search.cpp:563-570) is applied while loading.
// score: per sliding-box position, the occupied-voxel gate (exact integer box sum of
//   exist_voxel_num, = the reference's int summed-volume table), the box feature as a
//   direct sum of the box's subdivision vectors (no fp32 summed-volume differencing:
//   see DESIGN.md "A12"), then |Q_m f| / |f| per model with the reference's double
//   sqrt/divide.  Scores of gated-out positions are -1.
// replay: the order-dependent rank update with checkOverlap (search.cpp:327-376,
//   464-474) replayed exactly, one wave per model, scanning positions in the
//   reference's (mode, z, y, x) order; only candidates above the current rank-th score
//   (the lists only grow) are visited serially.
#include "c3h_internal.h"

namespace c3h {
namespace {

// ---------------------------------------------------------------- compress (GEMM)
// G[h][d] = sum_j f'[h][j] * P[j][d] (P = whitened axis_p transposed, F x Dpad).
// 512-thread block: 64 rows x 128 columns; lane = row (f staged k-major in LDS, read
// conflict-free), wave = 16 columns whose P values are wave-uniform scalar loads.
// fma chain in ascending j (the reference's GEMV order).
constexpr int kCM = 64, kCN = 128, kCK = 128, kCT = 512, kCW = 16;

__global__ __launch_bounds__(kCT) void compress_kernel(
    const float* __restrict__ feat, int64_t H, int F, const float* __restrict__ PT, int D,
    int Dpad, const float* __restrict__ fmax, int fmax_len, float* __restrict__ G,
    const int32_t* __restrict__ rows, const uint32_t* __restrict__ nrows,
    const int32_t* __restrict__ exist) {
  __shared__ float fs[kCK * (kCM + 1)];
  __shared__ int64_t s_row[kCM];
  const int tid = threadIdx.x;
  const int row = tid & (kCM - 1);
  const int cg = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t h0 = blockIdx.x * (int64_t)kCM;
  // sparse mode: this block's rows are rows[h0 .. h0+63] of the non-empty-row list
  // (G rows of empty subdivisions are left untouched; consumers gate them on exist)
  const int64_t nr = rows ? (int64_t)*nrows : H;
  if (h0 >= nr) return;
  if (tid < kCM) s_row[tid] = h0 + tid < nr ? (rows ? (int64_t)rows[h0 + tid] : h0 + tid) : -1;
  __syncthreads();
  const int c0 = blockIdx.y * kCN + cg * kCW;
  const bool active = c0 < D;
  float acc[kCW];
#pragma unroll
  for (int j = 0; j < kCW; ++j) acc[j] = 0.0f;
  for (int j0 = 0; j0 < F; j0 += kCK) {
    const int kn = min(kCK, F - j0);
    int r = tid / kn, c = tid - (tid / kn) * kn;  // e = tid + kCT*i -> (r, c), no division in the loop
    const int sr = kCT / kn, sc = kCT - (kCT / kn) * kn;
    for (int e = tid; e < kCM * kn; e += kCT) {
      const int64_t hh = s_row[r];
      const int jj = j0 + c;
      float v = 0.0f;
      // exist gate (sparse features: rows of empty subdivisions are stale, their true
      // value is 0, which is what an ungated zero row would give)
      if (hh >= 0 && (!exist || exist[hh])) {
        v = feat[hh * F + jj];
        if (jj < fmax_len) {  // SearchObj::setData histogram normalisation (search.cpp:563-570)
          const float mx = fmax[jj];
          if (mx == 0.0f) v = 0.0f;
          else if (v == mx) v = 1.0f;
          else v = __fdiv_rn(v, mx);
        }
      }
      fs[c * (kCM + 1) + r] = v;
      r += sr;
      c += sc;
      if (c >= kn) {
        c -= kn;
        ++r;
      }
    }
    __syncthreads();
    if (active) {
      const float* __restrict__ pk = PT + (int64_t)j0 * Dpad + c0;
      for (int k = 0; k < kn; ++k) {
        const float fv = fs[k * (kCM + 1) + row];
        const float* __restrict__ p = pk + (int64_t)k * Dpad;
#pragma unroll
        for (int j = 0; j < kCW; ++j) acc[j] = __builtin_fmaf(fv, p[j], acc[j]);
      }
    }
    __syncthreads();
  }
  const int64_t hh = s_row[row];
  if (active && hh >= 0) {
#pragma unroll
    for (int j = 0; j < kCW; ++j)
      if (c0 + j < D) G[hh * D + c0 + j] = acc[j];
  }
}

// Sparse compress (row list from the extract): 16 listed rows per workgroup x all
// columns (Dpad <= 128).  The 16 feature rows (max-normalised) and 32-row chunks of P
// are staged in LDS, P prefetched one chunk ahead into registers so only the first
// load's latency is exposed; thread = (row, 8 columns); the fma chain per output runs
// in ascending j exactly like compress_kernel, so both paths give identical G rows.
constexpr int kRR = 16, kRK = 32;
constexpr int kCompressGridCap = 128;  // row-block workgroups per frame of the fused launch

struct CompressRows {
  const float* feat;
  const float* PT;
  const float* fmax;
  float* G;
  const int32_t* rows;
  const uint32_t* nrows;
  int F, D, Dpad, fmax_len;
  int64_t s_feat, s_G, s_rows, s_nrows;  // per-frame strides (frame = launch y / z index)
};

__device__ __forceinline__ void compress_rows_body(const CompressRows& cr, int bid, int nblk, int64_t f) {
  const float* __restrict__ feat = cr.feat + f * cr.s_feat;
  const float* __restrict__ fmax = cr.fmax;
  float* __restrict__ G = cr.G + f * cr.s_G;
  const int32_t* __restrict__ rows = cr.rows + f * cr.s_rows;
  const int F = cr.F, D = cr.D, Dpad = cr.Dpad, fmax_len = cr.fmax_len;
  extern __shared__ __attribute__((aligned(16))) float csm[];
  float* pc = csm;                 // kRK x Dpad
  float* fs = csm + kRK * Dpad;    // kRR x F
  const int tid = threadIdx.x;
  const int nq4 = kRK * Dpad / 4, tot4 = F * Dpad / 4;
  const float4* P4 = reinterpret_cast<const float4*>(cr.PT);
  float4 pre[4];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + j * kBlock, g = c * nq4 + e;
      pre[j] = (e < nq4 && g < tot4) ? P4[g] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // P's first chunk is independent of the row count: in flight before the count arrives
  load_chunk(0);
  const int n = (int)cr.nrows[f * cr.s_nrows];
  const int row = tid >> 4, cg = tid & 15;
  const bool active = 8 * cg < Dpad;
  const int nch = (F + kRK - 1) / kRK;
  // row blocks bid, bid + nblk, ... (the launch holds few workgroups; dense scenes loop)
  for (int r0 = bid * kRR; r0 < n; r0 += nblk * kRR) {
    if (r0 != bid * kRR) load_chunk(0);
    for (int e = tid; e < kRR * F; e += kBlock) {
      const int r = e / F, j = e - r * F;
      float v = 0.0f;
      if (r0 + r < n) {
        v = feat[(int64_t)rows[r0 + r] * F + j];
        if (j < fmax_len) {  // setData max-normalisation (search.cpp:563-570)
          const float mx = fmax[j];
          if (mx == 0.0f) v = 0.0f;
          else if (v == mx) v = 1.0f;
          else v = __fdiv_rn(v, mx);
        }
      }
      fs[e] = v;
    }
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.0f;
    for (int c = 0; c < nch; ++c) {
      lds_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + j * kBlock;
        if (e < nq4) reinterpret_cast<float4*>(pc)[e] = pre[j];
      }
      if (c + 1 < nch) load_chunk(c + 1);
      lds_barrier();
      if (active) {
        const int kn = min(kRK, F - c * kRK);
        const float* fr = fs + row * F + c * kRK;
        for (int k = 0; k < kn; ++k) {
          const float fv = fr[k];
          const float4 p0 = *reinterpret_cast<const float4*>(&pc[k * Dpad + 8 * cg]);
          const float4 p1 = *reinterpret_cast<const float4*>(&pc[k * Dpad + 8 * cg + 4]);
          acc[0] = __builtin_fmaf(fv, p0.x, acc[0]);
          acc[1] = __builtin_fmaf(fv, p0.y, acc[1]);
          acc[2] = __builtin_fmaf(fv, p0.z, acc[2]);
          acc[3] = __builtin_fmaf(fv, p0.w, acc[3]);
          acc[4] = __builtin_fmaf(fv, p1.x, acc[4]);
          acc[5] = __builtin_fmaf(fv, p1.y, acc[5]);
          acc[6] = __builtin_fmaf(fv, p1.z, acc[6]);
          acc[7] = __builtin_fmaf(fv, p1.w, acc[7]);
        }
      }
    }
    if (active && r0 + row < n) {
      const int64_t h = rows[r0 + row];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (8 * cg + q < D) G[h * D + 8 * cg + q] = acc[q];
    }
    lds_barrier();  // fs / pc are rewritten by the next row block
  }
}

__global__ __launch_bounds__(kBlock) void compress_rows_kernel(CompressRows cr) {
  compress_rows_body(cr, blockIdx.x, gridDim.x, blockIdx.y);
}

// ---------------------------------------------------------------- score
// Generic path (any D, any M*r): SP positions per workgroup, basis through the scalar path.
template <int SP>
__global__ __launch_bounds__(kBlock) void score_kernel(ScoreLaunch a, int64_t P) {
  extern __shared__ __attribute__((aligned(16))) float ssm[];
  const int DP = a.D + 1;
  float* fbox = ssm;                  // SP x DP
  float* qv = fbox + SP * DP;         // r x SP
  float* ffv = qv + a.r * SP;         // SP
  int* gate = reinterpret_cast<int*>(ffv + SP);  // SP
  const int tid = threadIdx.x;
  const int64_t p0 = blockIdx.x * (int64_t)SP;
  const int xyn = a.xn * a.yn;

  if (tid < SP) {
    const int64_t p = p0 + tid;
    int ok = 0;
    if (p < P) {
      const int x = (int)(p % a.xe), y = (int)((p / a.xe) % a.ye), z = (int)(p / ((int64_t)a.xe * a.ye));
      int e = 0;
      for (int dz = 0; dz < a.zr; ++dz)
        for (int dy = 0; dy < a.yr; ++dy)
          for (int dx = 0; dx < a.xr; ++dx) e += a.exist[(z + dz) * xyn + (y + dy) * a.xn + x + dx];
      ok = e > a.thr;
    }
    gate[tid] = ok;
  }
  __syncthreads();
  for (int idx = tid; idx < SP * a.D; idx += kBlock) {
    const int pp = idx / a.D, d = idx - pp * a.D;
    float s = 0.0f;
    if (gate[pp]) {
      const int64_t p = p0 + pp;
      const int x = (int)(p % a.xe), y = (int)((p / a.xe) % a.ye), z = (int)(p / ((int64_t)a.xe * a.ye));
      for (int dz = 0; dz < a.zr; ++dz)
        for (int dy = 0; dy < a.yr; ++dy)
          for (int dx = 0; dx < a.xr; ++dx)
            s += a.G[(int64_t)((z + dz) * xyn + (y + dy) * a.xn + x + dx) * a.D + d];
    }
    fbox[pp * DP + d] = s;
  }
  __syncthreads();
  if (tid < SP) {
    float s = 0.0f;
    for (int d = 0; d < a.D; ++d) s = __builtin_fmaf(fbox[tid * DP + d], fbox[tid * DP + d], s);
    ffv[tid] = s;
  }
  constexpr int kRowsPerPass = kBlock / SP;
  const int pp = tid & (SP - 1);
  const int i0 = __builtin_amdgcn_readfirstlane(tid / SP);
  for (int m = 0; m < a.M; ++m) {
    const float* __restrict__ Q = a.axis_q + (int64_t)m * a.r * a.D;
    for (int i = i0; i < a.r; i += kRowsPerPass) {
      float t = 0.0f;
      const float* qrow = Q + (int64_t)i * a.D;
      const float* frow = fbox + pp * DP;
      for (int d = 0; d < a.D; ++d) t = __builtin_fmaf(qrow[d], frow[d], t);
      qv[i * SP + pp] = t;
    }
    __syncthreads();
    if (tid < SP) {
      const int64_t p = p0 + tid;
      if (p < P) {
        double sc = -1.0;
        if (gate[tid]) {
          float q2 = 0.0f;
          for (int i = 0; i < a.r; ++i) q2 = __builtin_fmaf(qv[i * SP + tid], qv[i * SP + tid], q2);
          sc = sqrt((double)q2) / sqrt((double)ffv[tid]);
        }
        a.scores[(int64_t)m * P + p] = sc;
      }
    }
    __syncthreads();
  }
}

// Fast path (D <= 256, D % 4 == 0, M*r <= 256) = the sparse search below: 32 list
// entries per workgroup.  Box features are summed with float4 loads and staged k-major in
// LDS (lanes = positions: conflict-free); the projection onto all M*r basis rows is a
// 32 x Opad x D fp32 GEMM with a 2-position x 16-row register tile per thread (one
// ds_read_b64 of box features + four ds_read_b128 of basis rows feed 32 FMAs), the basis
// streamed through LDS in 16-row chunks prefetched one chunk ahead into registers;
// |Q_m f|^2 is summed per (position, model) in a fixed order.  The block also emits its
// per-model best (score, scan order) so rank-1 searches need no second pass.
constexpr int kFP = 32;
constexpr int kOC = 64;  // basis rows per workgroup (whole models)
constexpr int kScoreGridCap = 128;  // workgroups per (model group, frame) of the score launch

// ---------------------------------------------------------------- sparse search
// The exist gate passes few positions on surface scenes (a depth camera sees a 2-D
// manifold), so the gate runs first over every position of every mode and compacts the
// passing ones into a list; the projection then runs over the list only.  Entries are
// (mode index << 40) | position; list order is irrelevant: scores are per position and
// the per-block partials break ties on the scan order explicitly.
// this frame's view of a batched search (per-frame buffers at base + f * stride)
__device__ __forceinline__ SparseSearch frame_view(const SparseSearch& b, int64_t f) {
  SparseSearch a = b;
  a.G = b.G + f * b.s_G;
  a.exist = b.exist + f * b.s_exist;
  a.scores = b.scores + f * b.s_scores;
  a.list = b.list + f * b.s_list;
  a.cnt = b.cnt + f * b.s_cnt;
  a.done = b.done + f * b.s_cnt;
  if (b.partials) a.partials = b.partials + f * b.s_partials;
  if (b.lists) a.lists = b.lists + f * b.s_lists;
  a.outs[0] = b.outs[f];
  if (f) a.prof = nullptr;
  return a;
}

__device__ __forceinline__ int find_mode(const SparseSearch& a, int64_t g) {
  int mi = 0;
  while (mi + 1 < a.nmodes && g >= a.pstart[mi + 1]) ++mi;
  return mi;
}

__device__ __forceinline__ void gate_body(const SparseSearch& a, int bid) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (bid == 0 && tid == 0) {  // the next search's counters
    a.cnt[(a.epoch + 1) & 1] = 0;
    a.done[(a.epoch + 1) & 1] = 0;
  }
  const int64_t g = bid * (int64_t)kBlock + tid;
  bool pass = false;
  int64_t entry = 0;
  if (g < a.pstart[a.nmodes]) {
    const int mi = find_mode(a, g);
    const ModeGeom& md = a.md[mi];
    const int64_t p = g - a.pstart[mi];
    const int64_t xye = (int64_t)md.xe * md.ye;
    const int x = (int)(p % md.xe), y = (int)((p / md.xe) % md.ye), z = (int)(p / xye);
    const int xyn = a.xn * a.yn;
    const int h = z * xyn + y * a.xn + x;
    int e = 0;  // SearchObj::clipValue<int> on exist_voxel_num (search.cpp:484-535), exact
    for (int dz = 0; dz < md.zr; ++dz)
      for (int dy = 0; dy < md.yr; ++dy)
        for (int dx = 0; dx < md.xr; ++dx) e += a.exist[h + dz * xyn + dy * a.xn + dx];
    pass = e > a.thr;
    entry = ((int64_t)mi << 40) | p;
    if (!pass)
      for (int m = 0; m < a.M; ++m) a.scores[md.offset + (int64_t)m * md.P + p] = -1.0;
  }
  const unsigned long long m = __ballot(pass);
  if (m) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&a.cnt[a.epoch & 1], (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (pass) a.list[base + __popcll(m & ((1ull << lane) - 1))] = entry;
  }
}

__global__ __launch_bounds__(kBlock) void gate_kernel(SparseSearch b) {
  gate_body(frame_view(b, blockIdx.y), blockIdx.x);
}

// one launch for two independent stages: gate workgroups first, then the sparse compress
__global__ __launch_bounds__(kBlock) void compress_gate_kernel(CompressRows cr, SparseSearch b, int ngate) {
  if ((int)blockIdx.x < ngate) gate_body(frame_view(b, blockIdx.y), blockIdx.x);
  else compress_rows_body(cr, blockIdx.x - ngate, gridDim.x - ngate, blockIdx.y);
}

// Rank-1 replay fused into the score launch (search.cpp:464-474 with rank_num == 1:
// checkOverlap returns slot 0, so the update is "first strictly greater maximum in scan
// order").  One wave per model reduces the partials with (score desc, scan order asc);
// partials of other workgroups are read with device-scope atomic loads.
__device__ void argmax_finalize(const SparseSearch& a, const ScorePartial* partials, c3h_det* lists,
                                c3h_det* out, int nparts) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int m = w; m < a.M; m += kBlock / 64) {
    double best = -2.0;
    long long bo = -1;
    for (int i = lane; i < nparts; i += 64) {
      const ScorePartial* q = partials + (int64_t)i * a.M + m;
      const long long qo = __hip_atomic_load(&q->order, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double qs = __hip_atomic_load(&q->score, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (qo >= 0 && (qs > best || (qs == best && qo < bo))) {
        best = qs;
        bo = qo;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double os = __shfl_xor(best, o, 64);
      const long long oo = __shfl_xor(bo, o, 64);
      if (oo >= 0 && (os > best || (os == best && (bo < 0 || oo < bo)))) {
        best = os;
        bo = oo;
      }
    }
    if (lane == 0) {
      c3h_det e = lists[m];
      if (a.clean) {  // 1: cleanMax (modes kept, search.cpp:683-690); 2: setRank state
        e.score = 0.0;
        e.x = e.y = e.z = 0;
        if (a.clean == 2) e.mode = 0;
      }
      if (bo >= 0 && best > e.score) {
        const int mi = (int)(bo >> 40);
        const int64_t p = bo & ((1ll << 40) - 1);
        const ModeGeom& md = a.md[mi];
        e.score = best;
        e.x = (int)(p % md.xe);
        e.y = (int)((p / md.xe) % md.ye);
        e.z = (int)(p / ((int64_t)md.xe * md.ye));
        e.mode = md.mode;
      }
      lists[m] = e;
      if (out) out[m] = e;
    }
  }
}

// Fast-path projection over the gate list:
// kFP entries per workgroup; box rows of empty subdivisions are skipped (their G rows
// may be stale: the sparse compress only writes non-empty rows; an all-zero row adds
// nothing to a sum that starts at +0).
__global__ __launch_bounds__(kBlock) void score_list_kernel(SparseSearch b) {
  const SparseSearch& a = b;  // frame-independent fields; per-frame pointers below
  const int64_t fz = blockIdx.z;
  const float* __restrict__ fG = b.G + fz * b.s_G;
  const int32_t* __restrict__ fexist = b.exist + fz * b.s_exist;
  double* __restrict__ fscores = b.scores + fz * b.s_scores;
  const long long* __restrict__ flist = b.list + fz * b.s_list;
  const uint32_t* fcnt = b.cnt + fz * b.s_cnt;
  uint32_t* fdone = b.done + fz * b.s_cnt;
  ScorePartial* fpart = b.partials ? b.partials + fz * b.s_partials : nullptr;
  c3h_det* flists = b.lists ? b.lists + fz * b.s_lists : nullptr;
  c3h_det* fout = b.outs[fz];
  long long* fprof = fz ? nullptr : b.prof;
  extern __shared__ __attribute__((aligned(16))) float ssm[];
  const int D = a.D, D4 = a.D >> 2, Qs = a.Opad;  // qt row stride
#define C3H_SPROF(k) \
  if (fprof && threadIdx.x == 0 && blockIdx.y == 0) fprof[blockIdx.x * 8 + (k)] = (long long)wall_clock64()
  C3H_SPROF(0);
  const int tid = threadIdx.x;
  // issued together: the list count, this workgroup's first list chunk (speculative: the
  // list buffer holds P_total entries, entries past the count are ignored) and the
  // group's basis window, so the count costs no extra round trip
  const int64_t ptot = a.pstart[a.nmodes];
  long long en_first = -1;
  if (tid < kFP) en_first = flist[min((int64_t)blockIdx.x * kFP + tid, ptot - 1)];
  // model group of this workgroup: models [m0, m1), basis rows [m0*r, m1*r) padded to oc
  const int m0 = blockIdx.y * a.mpg, m1 = min(a.M, m0 + a.mpg);
  const int row0 = m0 * a.r, oc = ((m1 - m0) * a.r + 15) & ~15;  // <= kOC
  constexpr int kQW = 160 * kOC / kBlock;  // window floats per lane at the largest D
  float qwv[kQW];
#pragma unroll
  for (int j = 0; j < kQW; ++j) {
    const int e = j * kBlock + tid, d = e / oc, o = e - d * oc;
    qwv[j] = e < D * oc ? a.qt[(int64_t)d * Qs + row0 + o] : 0.0f;
  }
  const int n = (int)fcnt[a.epoch & 1];
  const int nch = (n + kFP - 1) / kFP;  // list chunks; chunk c -> workgroups c mod gridDim.x
  if ((int)blockIdx.x >= nch) {
    if (n == 0 && flists && blockIdx.x == 0 && blockIdx.y == 0) argmax_finalize(a, fpart, flists, fout, 0);  // clean / copy out
    return;
  }
  const int fts = max(D * kFP, kFP * (kOC + 1));
  float* fT = ssm;                    // D x kFP (k-major box features)
  float* qv = ssm;                    // kFP x (kOC+1), aliases fT after the GEMM
  float* qw = ssm + fts;              // D x oc: this group's whole basis window
  float* ffv = qw + D * kOC;
  int* gate = reinterpret_cast<int*>(ffv + kFP);
  int* hrow = gate + kFP;
  int* rng = hrow + kFP;                       // packed xr | yr << 10 | zr << 20
  long long* ent = reinterpret_cast<long long*>(rng + kFP + (kFP & 1));
  double* bsc = reinterpret_cast<double*>(ent + kFP);  // kFP * mpg
  const int xyn = a.xn * a.yn;
#pragma unroll
  for (int j = 0; j < kQW; ++j)  // parked once; read by every chunk's GEMM
    if (j * kBlock + tid < D * oc) qw[j * kBlock + tid] = qwv[j];
  for (int ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int64_t e0 = (int64_t)ch * kFP;
    if (tid < kFP) {
      const int64_t e = e0 + tid;
      int ok = 0, h = 0, rr = 0;
      long long en = -1;
      if (e < n) {
        en = ch == (int)blockIdx.x ? en_first : flist[e];
        const int mi = (int)(en >> 40);
        const int64_t p = en & ((1ll << 40) - 1);
        const ModeGeom& md = a.md[mi];
        const int64_t xye = (int64_t)md.xe * md.ye;
        const int x = (int)(p % md.xe), y = (int)((p / md.xe) % md.ye), z = (int)(p / xye);
        h = z * xyn + y * a.xn + x;
        rr = md.xr | (md.yr << 10) | (md.zr << 20);
        ok = 1;
      }
      gate[tid] = ok;
      hrow[tid] = h;
      rng[tid] = rr;
      ent[tid] = en;
    }
    lds_barrier();
    C3H_SPROF(1);
    {  // box sums in the fixed (dz, dy, dx) order over non-empty rows; lane = position.
       // Cells go in batches of 4 x (this thread's d4 slots): every load of a batch is in
       // flight together.  Rows of empty subdivisions read as 0 (their G rows may be stale;
       // +0 added to a sum that starts at +0 changes nothing).
      const int pp = tid & (kFP - 1), dg = tid / kFP;
      constexpr int kDG = kBlock / kFP;  // d4 stride
      const bool ok = gate[pp];
      const int h = hrow[pp], rr = rng[pp];
      const int xr = rr & 1023, yr = (rr >> 10) & 1023, zr = rr >> 20;
      const int ncell = ok ? xr * yr * zr : 0;
      const float4* G4 = reinterpret_cast<const float4*>(fG);
      constexpr int kSlots = 4;  // d4 values per thread handled together (D4 <= 64)
      float4 s[kSlots];
#pragma unroll
      for (int q = 0; q < kSlots; ++q) s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int d4b = 0; d4b < D4; d4b += kSlots * kDG) {
        for (int c0 = 0; c0 < ncell; c0 += 4) {
          float4 g[4][kSlots];
          bool lv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = c0 + k;
            const int dx = c % xr, dy = (c / xr) % yr, dz = c / (xr * yr);
            const int hh = h + dz * xyn + dy * a.xn + dx;
            lv[k] = c < ncell && fexist[c < ncell ? hh : h] != 0;
#pragma unroll
            for (int q = 0; q < kSlots; ++q) {
              const int d4 = d4b + dg + q * kDG;
              g[k][q] = (c < ncell && d4 < D4) ? G4[(int64_t)hh * D4 + d4] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int q = 0; q < kSlots; ++q)
              if (lv[k]) {
                s[q].x += g[k][q].x;
                s[q].y += g[k][q].y;
                s[q].z += g[k][q].z;
                s[q].w += g[k][q].w;
              }
        }
#pragma unroll
        for (int q = 0; q < kSlots; ++q) {
          const int d4 = d4b + dg + q * kDG;
          if (d4 < D4) {
            fT[(4 * d4 + 0) * kFP + pp] = s[q].x;
            fT[(4 * d4 + 1) * kFP + pp] = s[q].y;
            fT[(4 * d4 + 2) * kFP + pp] = s[q].z;
            fT[(4 * d4 + 3) * kFP + pp] = s[q].w;
          }
          s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    lds_barrier();
    C3H_SPROF(2);
    if (tid < kFP) {
      float s = 0.0f;
      for (int d = 0; d < D; ++d) s = __builtin_fmaf(fT[d * kFP + tid], fT[d * kFP + tid], s);
      ffv[tid] = s;
    }
    // GEMM: thread (tp, to): positions 2*tp, 2*tp+1; basis rows 4*to .. 4*to+3 of the group
    const int tp = tid & 15, to = tid >> 4;
    const bool active = 4 * to < oc;
    float acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[i][q] = 0.0f;
    if (active) {
#pragma unroll 4
      for (int d = 0; d < D; ++d) {
        const float2 f = *reinterpret_cast<const float2*>(&fT[d * kFP + 2 * tp]);
        const float4 q = *reinterpret_cast<const float4*>(&qw[d * oc + 4 * to]);
        acc[0][0] = __builtin_fmaf(f.x, q.x, acc[0][0]);
        acc[0][1] = __builtin_fmaf(f.x, q.y, acc[0][1]);
        acc[0][2] = __builtin_fmaf(f.x, q.z, acc[0][2]);
        acc[0][3] = __builtin_fmaf(f.x, q.w, acc[0][3]);
        acc[1][0] = __builtin_fmaf(f.y, q.x, acc[1][0]);
        acc[1][1] = __builtin_fmaf(f.y, q.y, acc[1][1]);
        acc[1][2] = __builtin_fmaf(f.y, q.z, acc[1][2]);
        acc[1][3] = __builtin_fmaf(f.y, q.w, acc[1][3]);
      }
    }
    lds_barrier();  // qv aliases fT
    C3H_SPROF(3);
    if (active) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) qv[(2 * tp + i) * (kOC + 1) + 4 * to + q] = acc[i][q];
    }
    lds_barrier();
    const int nm = m1 - m0;
    for (int e = tid; e < kFP * nm; e += kBlock) {
      const int mm = e / kFP, pp = e - mm * kFP;
      double sc = -2.0;
      if (gate[pp]) {
        float q2 = 0.0f;
        const float* q = qv + pp * (kOC + 1) + mm * a.r;
        for (int i = 0; i < a.r; ++i) q2 = __builtin_fmaf(q[i], q[i], q2);
        sc = sqrt((double)q2) / sqrt((double)ffv[pp]);
        const long long en = ent[pp];
        const ModeGeom& md = a.md[(int)(en >> 40)];
        fscores[md.offset + (int64_t)(m0 + mm) * md.P + (en & ((1ll << 40) - 1))] = sc;
      }
      bsc[e] = sc;
    }
    C3H_SPROF(4);
    if (fpart) {
      lds_barrier();
      for (int mm = tid; mm < nm; mm += kBlock) {  // (score desc, scan order asc)
        double best = -2.0;
        long long bo = -1;
        for (int pp = 0; pp < kFP; ++pp) {
          if (!gate[pp]) continue;
          const double sc = bsc[mm * kFP + pp];
          const long long en = ent[pp];
          const long long o = a.order_base[(int)(en >> 40)] + (en & ((1ll << 40) - 1));
          if (sc > best || (sc == best && o < bo)) {
            best = sc;
            bo = o;
          }
        }
        ScorePartial* q = fpart + (int64_t)ch * a.M + m0 + mm;
        if (flists) {  // handed to another workgroup inside this launch: sc1 stores
          __hip_atomic_store(&q->score, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&q->order, bo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          *q = ScorePartial{best, bo};
        }
      }
    }
    lds_barrier();  // LDS is reused by the next chunk
  }
  if (fpart && flists) {
    // rank 1, fused replay: the last workgroup to finish reduces.  Hand-off per
    // MI355X_MICROARCH.md (inter-workgroup visibility, table row 1): sc1 stores, every
    // storing wave waits vmcnt(0), a barrier, one agent atomic add per workgroup; the
    // workgroup whose add returns total-1 reads the partials with sc1 loads.
    __shared__ int s_last;
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (tid == 0) {
      const uint32_t total = (uint32_t)min(nch, (int)gridDim.x) * gridDim.y;
      s_last = atomicAdd(&fdone[a.epoch & 1], 1u) == total - 1;
    }
    lds_barrier();
    if (s_last) argmax_finalize(a, fpart, flists, fout, nch);
  }
  C3H_SPROF(7);
}

// ---------------------------------------------------------------- rank replay
__device__ __forceinline__ void get_range(int mode, int r1, int r2, int r3, int& xr, int& yr,
                                          int& zr) {
  switch (mode) {  // search.cpp:218-251
    case 0: xr = r1; yr = r2; zr = r3; break;
    case 1: xr = r1; yr = r3; zr = r2; break;
    case 2: xr = r2; yr = r1; zr = r3; break;
    case 3: xr = r2; yr = r3; zr = r1; break;
    case 4: xr = r3; yr = r1; zr = r2; break;
    default: xr = r3; yr = r2; zr = r1; break;
  }
}

// rank update of searchPart (search.cpp:464-474) incl. checkOverlap (:327-356)
__device__ void rank_update(c3h_det* L, int rank, double cs, int x, int y, int z, int mode,
                            int xr, int yr, int zr, int r1, int r2, int r3) {
  for (int i = 0; i < rank; i++) {
    if (cs > L[i].score) {
      int num;
      for (num = 0; num < rank - 1; num++) {
        int oxr, oyr, ozr;
        get_range(L[num].mode, r1, r2, r3, oxr, oyr, ozr);
        int v1 = L[num].x - x;
        v1 = v1 < 0 ? -v1 - oxr : v1 - xr;
        int v2 = L[num].y - y;
        v2 = v2 < 0 ? -v2 - oyr : v2 - yr;
        int v3 = L[num].z - z;
        v3 = v3 < 0 ? -v3 - ozr : v3 - zr;
        if (v1 <= 0 && v2 <= 0 && v3 <= 0) break;
      }
      for (int q = 0; q < num - i; q++) L[num - q] = L[num - 1 - q];
      if (i <= num) {
        L[i].score = cs;
        L[i].x = x;
        L[i].y = y;
        L[i].z = z;
        L[i].mode = mode;
      }
      break;
    }
  }
}

// general rank: one wave per model scans the scores in (mode, z, y, x) order, eight
// 64-position chunks per load batch; only candidates above the current rank-th score
// (lists only grow) reach the serial update.
__global__ __launch_bounds__(64) void replay_kernel(const double* __restrict__ scores,
                                                    ReplayModes modes, int rank, int r1,
                                                    int r2, int r3, int clean,
                                                    c3h_det* __restrict__ lists,
                                                    c3h_det* __restrict__ out2) {
  extern __shared__ __attribute__((aligned(16))) c3h_det L[];
  const int m = blockIdx.x, lane = threadIdx.x;
  c3h_det* gl = lists + (int64_t)m * rank;
  for (int i = lane; i < rank; i += 64) {
    c3h_det e = gl[i];
    if (clean) {  // 1: cleanMax (modes kept); 2: setRank state
      e.score = 0.0;
      e.x = e.y = e.z = 0;
      if (clean == 2) e.mode = 0;
    }
    L[i] = e;
  }
  __syncthreads();
  for (int mi = 0; mi < modes.n; ++mi) {
    const ReplayMode md = modes.m[mi];
    int xr, yr, zr;
    get_range(md.mode, r1, r2, r3, xr, yr, zr);
    const double* sc = scores + md.offset + (int64_t)m * md.P;
    for (int64_t b0 = 0; b0 < md.P; b0 += 512) {
      double s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t p = b0 + 64 * j + lane;
        s[j] = p < md.P ? sc[p] : -1.0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t base = b0 + 64 * j;
        double T = L[rank - 1].score;
        unsigned long long mask = __ballot(s[j] > T);
        while (mask) {
          const int jl = __ffsll((long long)mask) - 1;
          const double cs = __shfl(s[j], jl, 64);
          if (lane == 0) {
            const int64_t pc = base + jl;
            rank_update(L, rank, cs, (int)(pc % md.xe), (int)((pc / md.xe) % md.ye),
                        (int)(pc / ((int64_t)md.xe * md.ye)), md.mode, xr, yr, zr, r1, r2, r3);
          }
          __syncthreads();
          T = L[rank - 1].score;
          const unsigned long long later = jl >= 63 ? 0ull : (~0ull << (jl + 1));
          mask = __ballot(s[j] > T) & later;
        }
      }
    }
  }
  __syncthreads();
  for (int i = lane; i < rank; i += 64) {
    gl[i] = L[i];
    if (out2) out2[(int64_t)m * rank + i] = L[i];
  }
}

}  // namespace

bool compress_rows_ok(int F, int Dpad) {
  return Dpad <= 128 && ((size_t)kRK * Dpad + (size_t)kRR * F) * 4 <= 65536;
}

hipError_t launch_compress(const float* feat, int64_t H, int F, const float* axis_pt, int D,
                           int Dpad, const float* fmax, int fmax_len, float* G,
                           const int32_t* rows, const uint32_t* nrows, const int32_t* exist,
                           hipStream_t s) {
  if (rows && compress_rows_ok(F, Dpad)) {  // sparse list
    const size_t lds = sizeof(float) * ((size_t)kRK * Dpad + (size_t)kRR * F);
    const CompressRows cr{feat, axis_pt, fmax, G, rows, nrows, F, D, Dpad, fmax_len, 0, 0, 0, 0};
    compress_rows_kernel<<<(unsigned)((H + kRR - 1) / kRR), kBlock, lds, s>>>(cr);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((H + kCM - 1) / kCM), (unsigned)((Dpad + kCN - 1) / kCN));
  compress_kernel<<<grid, kCT, 0, s>>>(feat, H, F, axis_pt, D, Dpad, fmax, fmax_len, G, rows, nrows, exist);
  return hipGetLastError();
}

// dst[h][:] = exist[h] ? src[h][:] : 0 (readback of sparse feature / G buffers)
__global__ __launch_bounds__(kBlock) void masked_rows_kernel(const float* __restrict__ src,
                                                             const int32_t* __restrict__ exist,
                                                             int64_t H, int W, float* __restrict__ dst) {
  const int64_t n = H * W;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int64_t h = i / W;
    dst[i] = exist[h] ? src[i] : 0.0f;
  }
}

hipError_t launch_masked_rows(const float* src, const int32_t* exist, int64_t H, int W, float* dst,
                              hipStream_t s) {
  const int64_t n = H * W;
  if (n <= 0) return hipSuccess;
  const unsigned g = (unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 4096);
  masked_rows_kernel<<<g, kBlock, 0, s>>>(src, exist, H, W, dst);
  return hipGetLastError();
}

size_t score_lds_bytes(int D, int r, int SP) {
  return sizeof(float) * ((size_t)SP * (D + 1) + (size_t)r * SP + SP) + sizeof(int) * SP;
}

bool score_fast_ok(int D, int r) { return D <= 160 && (D & 3) == 0 && r <= kOC; }

int64_t score_blocks(const ScoreLaunch& a) {
  const int64_t P = (int64_t)a.xe * a.ye * a.ze;
  if (score_fast_ok(a.D, a.r)) return (P + kFP - 1) / kFP;
  return a.D <= 256 ? (P + 63) / 64 : (P + 15) / 16;
}

hipError_t launch_score(const ScoreLaunch& a, hipStream_t s) {
  const int64_t P = (int64_t)a.xe * a.ye * a.ze;
  if (P <= 0) return hipSuccess;
  if (score_fast_ok(a.D, a.r)) {
    return hipErrorInvalidValue;  // the fast path is the sparse search (launch_sparse_search)
  } else if (a.D <= 256) {
    score_kernel<64><<<(unsigned)((P + 63) / 64), kBlock, score_lds_bytes(a.D, a.r, 64), s>>>(a, P);
  } else {
    score_kernel<16><<<(unsigned)((P + 15) / 16), kBlock, score_lds_bytes(a.D, a.r, 16), s>>>(a, P);
  }
  return hipGetLastError();
}

int64_t sparse_score_blocks(const SparseSearch& a) { return (a.pstart[a.nmodes] + kFP - 1) / kFP; }

hipError_t launch_sparse_search(const SparseSearch& a, const SparseCompress* sc, hipStream_t s) {
  const int64_t ptot = a.pstart[a.nmodes];
  if (ptot <= 0) return hipSuccess;
  const unsigned ngate = (unsigned)((ptot + kBlock - 1) / kBlock);
  const unsigned nf = (unsigned)a.nframes;
  if (sc) {  // compress (non-empty rows) and gate in one launch
    const CompressRows cr{sc->feat, sc->PT, sc->fmax, sc->G, sc->rows, sc->nrows, sc->F, sc->D, sc->Dpad,
                          sc->fmax_len, sc->s_feat, sc->s_G, sc->s_rows, sc->s_nrows};
    const size_t lds = sizeof(float) * ((size_t)kRK * sc->Dpad + (size_t)kRR * sc->F);
    // compress workgroups: surface frames have ~700 non-empty rows (~44 row blocks)
    const unsigned ncomp = (unsigned)std::min<int64_t>((sc->H + kRR - 1) / kRR, kCompressGridCap);
    compress_gate_kernel<<<dim3(ngate + ncomp, nf), kBlock, lds, s>>>(cr, a, (int)ngate);
  } else {
    gate_kernel<<<dim3(ngate, nf), kBlock, 0, s>>>(a);
  }
  const size_t region = std::max((size_t)a.D * kFP, (size_t)kFP * (kOC + 1)) + (size_t)a.D * kOC;
  const size_t lds = sizeof(float) * (region + kFP) + sizeof(int) * 4 * kFP + sizeof(long long) * kFP +
                     sizeof(double) * kFP * a.mpg + 16;
  const unsigned groups = (unsigned)((a.M + a.mpg - 1) / a.mpg);
  // workgroups per (group, frame): list chunks beyond the cap loop (dense scenes only);
  // surface frames pass ~1k positions (~30 chunks), so few workgroups exit unused
  const unsigned gx = (unsigned)std::min<int64_t>(sparse_score_blocks(a), kScoreGridCap);
  score_list_kernel<<<dim3(gx, groups, nf), kBlock, lds, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_replay(const double* scores, const ReplayModes& modes, int M, int rank,
                         int r1, int r2, int r3, int clean, c3h_det* lists, c3h_det* out2,
                         hipStream_t s) {
  replay_kernel<<<M, 64, sizeof(c3h_det) * rank, s>>>(scores, modes, rank, r1, r2, r3, clean,
                                                      lists, out2);
  return hipGetLastError();
}


}  // namespace c3h

// search2_dev.h -- lane-per-item bodies of the sparse search stages (compress rows and
// list scoring), the defaults wherever they apply (compress2_ok / score2_ok).
//
// Both stages are small GEMMs whose weights are tiny and shared by every item: the
// whitened compress axis P (F x Dpad) and the model basis qt (D x Opad).  Here a lane
// owns one item (a feature row, a box position), its operand column is staged k-major in
// LDS (conflict-free: lane = column), and each wave owns a 32/64-column slice of the
// outputs.  The weights are laid out per wave slice at setup (PW: F x 4 x 32, QW: D x 4 x
// 64, zero padded) and streamed through LDS in 8-row chunks, prefetched one chunk ahead
// into registers; every lane of a wave reads the same weights (ds_read_b128 broadcast),
// so 16 B of LDS feed 4 FMAs per lane and one read of the item column feeds 32/64.  The fma
// chains run in the same ascending order as the block bodies in search_dev.h (ascending
// j for G, ascending d for the projection, ascending basis row for |Q_m f|^2), so the
// results are bit-identical to them.  Loads whose lanes may be out of range use clamped
// addresses and a select after the load (a per-element "load or zero" makes hipcc branch
// around each load and serialise them).
#pragma once
#include <cstdint>

#include "search_dev.h"

namespace c3h {

constexpr int kWChunk = 8;  // weight rows per LDS chunk

// ---------------------------------------------------------------- compress, lane = row
constexpr int kC2Rows = 64;  // feature rows per workgroup round (one per lane)
constexpr int kC2Cols = 32;  // output columns per wave (register tile)
constexpr int kC2W = 4 * kC2Cols;  // PW row: the four waves' column slices

__host__ __device__ inline bool compress2_ok(int F, int D) { return F <= 160 && D <= 4 * kC2Cols; }
__host__ __device__ inline size_t compress2_lds_bytes(int F) {
  return sizeof(float) * ((size_t)F * (kC2Rows + 1) + (size_t)kWChunk * kC2W);
}
// PW[j][w][c] = P[j][w * cpw + c] (c < cpw and w * cpw + c < D, else 0), cpw = ceil(D/4)
inline void compress2_pack(const float* PT, int F, int D, int Dpad, float* PW) {
  const int cpw = (D + 3) / 4;
  for (int j = 0; j < F; ++j)
    for (int w = 0; w < 4; ++w)
      for (int c = 0; c < kC2Cols; ++c) {
        const int col = w * cpw + c;
        PW[((size_t)j * 4 + w) * kC2Cols + c] = (c < cpw && col < D) ? PT[(size_t)j * Dpad + col] : 0.0f;
      }
}

// G[h][c] = sum_j f'[h][j] P[j][c] for the listed rows h (rows[0 .. nrows)); workgroup
// bid of nblk takes row blocks bid, bid + nblk, ...; wave w the columns [w*cpw, w*cpw+cpw)
// with cpw = ceil(D / 4), weights from PW (compress2_pack).
__device__ __forceinline__ void compress2_body(const CompressRows& cr, int bid, int nblk, int64_t f, float* fs) {
  const float* __restrict__ feat = cr.feat + f * cr.s_feat;
  const float* __restrict__ fmax = cr.fmax;
  float* __restrict__ G = cr.G + f * cr.s_G;
  const int32_t* __restrict__ rows = cr.rows + f * cr.s_rows;
  const int F = cr.F, D = cr.D, fmax_len = cr.fmax_len;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cpw = (D + 3) >> 2, c0 = wave * cpw;
  const int n = (int)cr.nrows[f * cr.s_nrows];
  float* ws = fs + (size_t)F * (kC2Rows + 1);  // kWChunk x kC2W weight chunk
  for (int r0 = bid * kC2Rows; r0 < n; r0 += nblk * kC2Rows) {
    // stage the rows k-major (fs[j][row]), max-normalised (search.cpp:563-570)
    for (int e = tid; e < kC2Rows * F; e += kBlock) {
      const int r = e / F, j = e - r * F;
      const bool in = r0 + r < n;
      float v = feat[(int64_t)rows[in ? r0 + r : r0] * F + j];
      if (!in) v = 0.0f;
      if (j < fmax_len) {
        const float mx = fmax[j];
        if (mx == 0.0f) v = 0.0f;
        else if (v == mx) v = 1.0f;
        else v = __fdiv_rn(v, mx);
      }
      fs[j * (kC2Rows + 1) + r] = v;
    }
    lds_barrier();
    float acc[kC2Cols];
#pragma unroll
    for (int c = 0; c < kC2Cols; ++c) acc[c] = 0.0f;
    // PW chunks of kWChunk rows (kWChunk * kC2W floats = one float4 per thread)
    const float4* __restrict__ PW4 = reinterpret_cast<const float4*>(cr.PW);
    float4* ws4 = reinterpret_cast<float4*>(ws);
    const int nck = (F + kWChunk - 1) / kWChunk, tot4 = F * kC2W / 4;
    static_assert(kWChunk * kC2W / 4 == kBlock, "one float4 per thread per chunk");
    float4 pre = PW4[min(tid, tot4 - 1)];
    for (int ck = 0; ck < nck; ++ck) {
      lds_barrier();  // the previous chunk's readers are done
      ws4[tid] = pre;
      if (ck + 1 < nck) pre = PW4[min((ck + 1) * kBlock + tid, tot4 - 1)];
      lds_barrier();
      const int j0 = ck * kWChunk, jn = min(kWChunk, F - j0);
      for (int jj = 0; jj < jn; ++jj) {
        const float fv = fs[(j0 + jj) * (kC2Rows + 1) + lane];
        const float4* pw = ws4 + (jj * kC2W + wave * kC2Cols) / 4;
#pragma unroll
        for (int c4 = 0; c4 < kC2Cols / 4; ++c4) {
          const float4 q = pw[c4];
          acc[4 * c4 + 0] = __builtin_fmaf(fv, q.x, acc[4 * c4 + 0]);
          acc[4 * c4 + 1] = __builtin_fmaf(fv, q.y, acc[4 * c4 + 1]);
          acc[4 * c4 + 2] = __builtin_fmaf(fv, q.z, acc[4 * c4 + 2]);
          acc[4 * c4 + 3] = __builtin_fmaf(fv, q.w, acc[4 * c4 + 3]);
        }
      }
    }
    if (r0 + lane < n) {
      const int64_t h = rows[r0 + lane];
#pragma unroll
      for (int c = 0; c < kC2Cols; ++c)
        if (c < cpw && c0 + c < D) G[h * D + c0 + c] = acc[c];
    }
    lds_barrier();  // fs is restaged by the next row block
  }
}

// ---------------------------------------------------------------- scoring, lane = position
constexpr int kSP = 64;     // list entries (box positions) per chunk, one per lane
constexpr int kSRows = 64;  // basis rows per wave (whole models)
constexpr int kSW = 4 * kSRows;  // QW row: the four waves' basis windows

__host__ __device__ inline int score2_models_per_wave(int M) { return (M + 3) >> 2; }
__host__ __device__ inline bool score2_ok(int D, int M, int r) {
  return D <= 160 && (D & 3) == 0 && score2_models_per_wave(M) * r <= kSRows;
}
__host__ __device__ inline size_t score2_lds_bytes(int D) {
  return sizeof(float) * ((size_t)D * kSP + (size_t)kWChunk * kSW) + sizeof(int) * 3 * kSP +
         sizeof(long long) * kSP + 16;
}
// QW[d][w][i] = axis_q[m][i'][d] for wave w's models m = w*mpw + i / r, i' = i % r (i < mpw*r,
// m < M), else 0
inline void score2_pack(const float* axis_q, int M, int r, int D, float* QW) {
  const int mpw = score2_models_per_wave(M);
  for (int d = 0; d < D; ++d)
    for (int w = 0; w < 4; ++w)
      for (int i = 0; i < kSRows; ++i) {
        const int m = w * mpw + i / r;
        const bool in = i < mpw * r && m < M;
        QW[((size_t)d * 4 + w) * kSRows + i] = in ? axis_q[((size_t)m * r + i % r) * D + d] : 0.0f;
      }
}
__host__ __device__ inline int64_t score2_chunks(int64_t entries) { return (entries + kSP - 1) / kSP; }

// workgroup bx of gdx for frame fz; smem: score2_lds_bytes(D).  Chunk ch of the gate list
// -> workgroups ch mod gdx.  Per chunk: box sums (fixed (dz, dy, dx) order over non-empty
// rows) into fT[d][lane]; wave w projects onto models [w*mpw, w*mpw + mpw); per
// (position, model) |Q f|^2 and the reference's double sqrt / divide; per model the
// chunk's best (score desc, scan order asc) by a wave reduction; rank 1: the last
// workgroup to finish reduces the partials into the lists (argmax_finalize).
__device__ __forceinline__ void score2_body(const SparseSearch& a, int bx, int fz_, int gdx, float* ssm) {
  const int64_t fz = fz_;
  const float* __restrict__ fG = a.G + fz * a.s_G;
  const int32_t* __restrict__ fexist = a.exist + fz * a.s_exist;
  double* __restrict__ fscores = a.scores + fz * a.s_scores;
  const long long* __restrict__ flist = a.list + fz * a.s_list;
  const uint32_t* fcnt = a.cnt + fz * a.s_cnt;
  uint32_t* fdone = a.done + fz * a.s_cnt;
  ScorePartial* fpart = a.partials ? a.partials + fz * a.s_partials : nullptr;
  c3h_det* flists = a.lists ? a.lists + fz * a.s_lists : nullptr;
  c3h_det* fout = a.outs[fz];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int D = a.D, D4 = a.D >> 2;
  const int n = (int)fcnt[a.epoch & 1];
  const int nch = (n + kSP - 1) / kSP;
  if (bx >= nch) {
    if (n == 0 && flists && bx == 0) argmax_finalize(a, fpart, flists, fout, 0);  // clean / copy out
    return;
  }
  float* fT = ssm;                                           // D x kSP
  float* qs = fT + (size_t)D * kSP;                          // kWChunk x kSW basis chunk
  int* okv = reinterpret_cast<int*>(qs + (size_t)kWChunk * kSW);  // kSP
  int* hrow = okv + kSP;
  int* rng = hrow + kSP;                                     // packed xr | yr << 10 | zr << 20
  long long* ent = reinterpret_cast<long long*>(rng + kSP);
  const int mpw = score2_models_per_wave(a.M);
  const int mw0 = wave * mpw, mw1 = min(a.M, mw0 + mpw);
  const int xyn = a.xn * a.yn;
  for (int ch = bx; ch < nch; ch += gdx) {
    if (tid < kSP) {
      const int64_t e = (int64_t)ch * kSP + tid;
      int ok = 0, h = 0, rr = 0;
      long long en = flist[e < n ? e : (int64_t)n - 1];
      if (e < n) {
        const int mi = (int)(en >> 40);
        const int64_t p = en & ((1ll << 40) - 1);
        const ModeGeom& md = a.md[mi];
        const int64_t xye = (int64_t)md.xe * md.ye;
        const int x = (int)(p % md.xe), y = (int)((p / md.xe) % md.ye), z = (int)(p / xye);
        h = z * xyn + y * a.xn + x;
        rr = md.xr | (md.yr << 10) | (md.zr << 20);
        ok = 1;
      } else {
        en = -1;
      }
      okv[tid] = ok;
      hrow[tid] = h;
      rng[tid] = rr;
      ent[tid] = en;
    }
    lds_barrier();
    {  // box sums; thread (lane = position, wave = d4 group), cells in batches of 4 with
       // every load of a batch in flight; rows of empty subdivisions read as 0
      constexpr int kDG = kBlock / kSP;
      constexpr int kSlots = 4;
      const bool ok = okv[lane];
      const int h = hrow[lane], rr = rng[lane];
      const int xr = rr & 1023, yr = (rr >> 10) & 1023, zr = rr >> 20;
      const int ncell = ok ? xr * yr * zr : 0;
      const float4* G4 = reinterpret_cast<const float4*>(fG);
      for (int d4b = 0; d4b < D4; d4b += kSlots * kDG) {
        float4 s[kSlots];
#pragma unroll
        for (int q = 0; q < kSlots; ++q) s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int c0 = 0; c0 < ncell; c0 += 4) {
          float4 g[4][kSlots];
          bool lv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = c0 + k;
            const int dx = c % xr, dy = (c / xr) % yr, dz = c / (xr * yr);
            const int hh = c < ncell ? h + dz * xyn + dy * a.xn + dx : h;
            lv[k] = c < ncell && fexist[hh] != 0;
#pragma unroll
            for (int q = 0; q < kSlots; ++q) {
              const int d4 = d4b + wave + q * kDG;
              const int64_t gi = (int64_t)hh * D4 + (d4 < D4 ? d4 : 0);
              g[k][q] = G4[gi];
              if (d4 >= D4) g[k][q] = make_float4(0.f, 0.f, 0.f, 0.f);
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
          const int d4 = d4b + wave + q * kDG;
          if (d4 < D4) {
            fT[(4 * d4 + 0) * kSP + lane] = s[q].x;
            fT[(4 * d4 + 1) * kSP + lane] = s[q].y;
            fT[(4 * d4 + 2) * kSP + lane] = s[q].z;
            fT[(4 * d4 + 3) * kSP + lane] = s[q].w;
          }
        }
      }
    }
    lds_barrier();
    {  // projection: lane = position, this wave's basis window (QW chunks through LDS)
      float acc[kSRows];
#pragma unroll
      for (int i = 0; i < kSRows; ++i) acc[i] = 0.0f;
      float ff = 0.0f;
      const float4* __restrict__ QW4 = reinterpret_cast<const float4*>(a.qw);
      float4* qs4 = reinterpret_cast<float4*>(qs);
      constexpr int kPer = kWChunk * kSW / 4 / kBlock;  // float4 per thread per chunk
      const int nck = (D + kWChunk - 1) / kWChunk, tot4 = D * kSW / 4;
      float4 pre[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) pre[j] = QW4[min(j * kBlock + tid, tot4 - 1)];
      for (int ck = 0; ck < nck; ++ck) {
        lds_barrier();  // the previous chunk's readers are done
#pragma unroll
        for (int j = 0; j < kPer; ++j) qs4[j * kBlock + tid] = pre[j];
        if (ck + 1 < nck)
#pragma unroll
          for (int j = 0; j < kPer; ++j) pre[j] = QW4[min((ck + 1) * kWChunk * kSW / 4 + j * kBlock + tid, tot4 - 1)];
        lds_barrier();
        if (mw0 < mw1) {
          const int d0 = ck * kWChunk, dn = min(kWChunk, D - d0);
          for (int dd = 0; dd < dn; ++dd) {
            const float f = fT[(d0 + dd) * kSP + lane];
            ff = __builtin_fmaf(f, f, ff);
            const float4* qw = qs4 + (dd * kSW + wave * kSRows) / 4;
#pragma unroll
            for (int i4 = 0; i4 < kSRows / 4; ++i4) {
              const float4 q = qw[i4];
              acc[4 * i4 + 0] = __builtin_fmaf(f, q.x, acc[4 * i4 + 0]);
              acc[4 * i4 + 1] = __builtin_fmaf(f, q.y, acc[4 * i4 + 1]);
              acc[4 * i4 + 2] = __builtin_fmaf(f, q.z, acc[4 * i4 + 2]);
              acc[4 * i4 + 3] = __builtin_fmaf(f, q.w, acc[4 * i4 + 3]);
            }
          }
        }
      }
      const bool ok = okv[lane];
      const long long en = ent[lane];
      const int mi = ok ? (int)(en >> 40) : 0;
      const int64_t p = en & ((1ll << 40) - 1);
      const ModeGeom& md = a.md[mi];
      const long long order = ok ? a.order_base[mi] + p : -1;
      for (int m = mw0; m < mw1; ++m) {  // (no iterations on waves without models)
        const int i0 = (m - mw0) * a.r, i1 = i0 + a.r;
        float q2 = 0.0f;
#pragma unroll
        for (int i = 0; i < kSRows; ++i) {  // this model's rows in ascending order (others add +0)
          const float v = (i >= i0 && i < i1) ? acc[i] : 0.0f;
          q2 = __builtin_fmaf(v, v, q2);
        }
        double best = -2.0;
        long long bo = -1;
        if (ok) {
          best = sqrt((double)q2) / sqrt((double)ff);
          bo = order;
          fscores[md.offset + (int64_t)m * md.P + p] = best;
        }
        if (fpart) {  // the chunk's best for model m: (score desc, scan order asc)
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            const double os = __shfl_xor(best, o, 64);
            const long long oo = __shfl_xor(bo, o, 64);
            if (oo >= 0 && (bo < 0 || os > best || (os == best && oo < bo))) {
              best = os;
              bo = oo;
            }
          }
          if (lane == 0) {
            ScorePartial* qp = fpart + (int64_t)ch * a.M + m;
            if (flists) {  // handed to another workgroup inside this launch: sc1 stores
              __hip_atomic_store(&qp->score, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(&qp->order, bo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              *qp = ScorePartial{best, bo};
            }
          }
        }
      }
    }
    lds_barrier();  // LDS is reused by the next chunk
  }
  if (fpart && flists) {
    // rank 1, fused replay: the last workgroup to finish reduces (hand-off as in
    // score_list_body: sc1 stores, every storing wave waits vmcnt(0), a barrier, one agent
    // atomic add per workgroup, sc1 loads in argmax_finalize)
    int& s_last = *reinterpret_cast<int*>(reinterpret_cast<char*>(ssm) + score2_lds_bytes(D) - 16);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (tid == 0) {
      const uint32_t total = (uint32_t)min(nch, gdx);
      s_last = atomicAdd(&fdone[a.epoch & 1], 1u) == total - 1;
    }
    lds_barrier();
    if (s_last) argmax_finalize(a, fpart, flists, fout, nch);
  }
}

}  // namespace c3h

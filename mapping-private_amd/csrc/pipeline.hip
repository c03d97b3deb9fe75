// pipeline.hip -- the software-pipelined "tick" kernel of c3h_run_frames.
//
// A frame batch goes through four dependent stages: occupancy stream (HBM-bound),
// C3 tile pass, sparse compress + exist gate, list scoring with the fused rank-1 argmax
// (all latency-bound).  Launched back to back per batch, or on parallel streams that
// drift into lock-step, the HBM stream idles while the latency-bound stages run.  Here
// every launch is one pipeline tick that hosts all four stages of four different batches
// as block roles:
//
//   tick t:  score(batch t-3) | compress+gate(t-2) | tile(t-1) | occupancy(t)
//
// Dependencies run only from one tick to the next (stream order), so no workgroup ever
// waits on another role; the batches use four rotating buffer sets (c3h_ctx lanes).
// Roles are dispatched occupancy first (one streaming workgroup per CU from the first
// cycle), then scoring, tile and compress+gate in the remaining workgroup slots: the score
// role's workgroups are the longest chains (one per list chunk running every model group),
// dispatched last they started ~550 us into a 64-frame tick and set its end; dispatched
// second they finish under the stream (profiles/r3/tick_order/: frac 0.662 -> 0.693).
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "c3hlac_dev.h"
#include "search_dev.h"

namespace c3h {
namespace {

struct TickArgs {
  int n_score, n_cg, n_tile, n_occ;  // workgroups per role (all frames of its batch)
  SparseSearch sq;                   // score role
  int s_gx, s_groups;
  SparseSearch gq;                   // compress + gate role
  CompressRows cr;
  int g_ngate, g_ncomp;
  int comp_mfma;                     // compress role on the matrix cores (compress_f32t_body)
  KArgs ka;                          // tile role
  int t_grid;
  OccArgs oa;                        // occupancy role
  int o_grid;
  int order;                         // role ids in dispatch order, 4 bits each (first in the low bits)
  int xcd;                           // bit r: role r keeps each frame's workgroups on one XCD
  long long* prof;                   // diagnostics (C3H_TICK_PROF): [block][2] start, end
};

// Workgroups of a role occupy one consecutive block range; t.order lists the role ids
// (0 occupancy, 1 tile, 2 compress+gate, 3 score) first-dispatched first.  The block index
// is mapped to the canonical layout (occupancy, tile, compress+gate, score) first, so the
// role bodies below see one fixed layout.
__device__ __forceinline__ int tick_canonical_block(const TickArgs& t) {
  const int n[4] = {t.n_occ, t.n_tile, t.n_cg, t.n_score};
  int b = blockIdx.x;
  for (int i = 0; i < 4; ++i) {
    const int r = (t.order >> (4 * i)) & 15;
    if (b < n[r]) {
      for (int k = 0; k < r; ++k) b += n[k];
      return b;
    }
    b -= n[r];
  }
  return b;
}

// wave priorities per role (s_setprio; 0 = the default): the arbiter of a SIMD picks the
// highest-priority ready wave.  The stream is the tick's critical path once the chains
// finish under it: its waves at priority 3 give +0.5 % (profiles/r3/tick_prio2/)
#ifndef C3H_TICK_PRIO_OCC
#define C3H_TICK_PRIO_OCC 3
#endif
#ifndef C3H_TICK_PRIO_TILE
#define C3H_TICK_PRIO_TILE 0
#endif
#ifndef C3H_TICK_PRIO_CG
#define C3H_TICK_PRIO_CG 0
#endif
#ifndef C3H_TICK_PRIO_SCORE
#define C3H_TICK_PRIO_SCORE 0
#endif
#define C3H_SETPRIO(p) \
  if constexpr ((p) > 0) __builtin_amdgcn_s_setprio(p)

// role-local block b -> (frame, block of that frame) for g blocks per frame.  XCD-placed:
// blocks b and b + 8 share an XCD under the observed round-robin dispatch (speed only, never
// correctness), so frame f takes the blocks with b % 8 == f % 8 -- every role of a frame
// then runs on one XCD tick after tick: halo rows shared by neighbouring tiles and the rows
// the next role re-reads (features, compressed rows) can be found in that XCD's L2
__device__ __forceinline__ void role_frame(int b, int g, bool xcd, int& f, int& local) {
  if (xcd) {
    const int q = b >> 3, k = q / g;
    f = (b & 7) + 8 * k;
    local = q - k * g;
  } else {
    f = b / g;
    local = b - f * g;
  }
}

__device__ __forceinline__ void tick_roles(const TickArgs& t, uint32_t* tick_smem) {
  int b = t.order == 0x3210 ? (int)blockIdx.x : tick_canonical_block(t);
  int f, r;
  if (b < t.n_occ) {
    C3H_SETPRIO(C3H_TICK_PRIO_OCC);
    role_frame(b, t.o_grid, t.xcd & 1, f, r);
    occupancy_bits_body<true>(t.oa, r, f, t.o_grid, tick_smem);
    return;
  }
  b -= t.n_occ;
  if (b < t.n_tile) {
    C3H_SETPRIO(C3H_TICK_PRIO_TILE);
    role_frame(b, t.t_grid, t.xcd & 2, f, r);
    if (t.ka.wave117) c3hlac_wave117_body(t.ka, r, f, t.t_grid, tick_smem);
    else c3hlac_tile_body(t.ka, r, f, t.t_grid, tick_smem);
    return;
  }
  b -= t.n_tile;
  if (b < t.n_cg) {
    C3H_SETPRIO(C3H_TICK_PRIO_CG);
    role_frame(b, t.g_ngate + t.g_ncomp, t.xcd & 4, f, r);
    if (r < t.g_ngate) gate_body(t.gq, r, f);
    else if (t.comp_mfma) compress_f32t_body(t.cr, r - t.g_ngate, t.g_ncomp, f, reinterpret_cast<float*>(tick_smem));
    else compress_rows_body(t.cr, r - t.g_ngate, t.g_ncomp, f, reinterpret_cast<float*>(tick_smem));
    return;
  }
  b -= t.n_cg;
  C3H_SETPRIO(C3H_TICK_PRIO_SCORE);
  role_frame(b, t.s_gx * t.s_groups, t.xcd & 8, f, r);
  score_list_body(t.sq, r % t.s_gx, r / t.s_gx, f, t.s_gx, t.s_groups, reinterpret_cast<float*>(tick_smem));
}

// waves per SIMD the register allocation must allow (4: the 128-VGPR cap); diagnostics builds
// try more resident workgroups per CU (tools/build_variant.sh NAME -DC3H_TICK_MINW=5)
#ifndef C3H_TICK_MINW
#define C3H_TICK_MINW 4
#endif
__global__ __launch_bounds__(kBlock, C3H_TICK_MINW) void c3h_tick_kernel(TickArgs t) {
  extern __shared__ __attribute__((aligned(16))) uint32_t tick_smem[];
  if (t.prof && threadIdx.x == 0) t.prof[2 * blockIdx.x] = (long long)wall_clock64();
  tick_roles(t, tick_smem);
  if (t.prof) {
    __syncthreads();
    if (threadIdx.x == 0) t.prof[2 * blockIdx.x + 1] = (long long)wall_clock64();
  }
}

// diagnostics (env C3H_TICK_PROF=<file>): per tick and role, block start/end spread in
// microseconds (wall_clock64: 100 MHz) from the tick's first block start.  Synchronises.
void tick_prof_dump(const TickArgs& t, long long* d_prof, int total, hipStream_t s) {
  std::vector<long long> v((size_t)2 * total);
  if (hipMemcpyAsync(v.data(), d_prof, v.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess) return;
  if (hipStreamSynchronize(s) != hipSuccess) return;
  FILE* fp = fopen(diag_env("C3H_TICK_PROF"), "a");
  if (!fp) return;
  long long t0 = LLONG_MAX;
  for (int b = 0; b < total; ++b) t0 = std::min(t0, v[2 * b]);
  const int n[4] = {t.n_occ, t.n_tile, t.n_cg, t.n_score};
  const char* names[4] = {"occ", "tile", "cg", "score"};
  int b0 = 0;
  fprintf(fp, "tick");
  for (int i = 0; i < 4; ++i) {
    const int r = (t.order >> (4 * i)) & 15;
    if (n[r]) {
      long long smin = LLONG_MAX, smax = 0, emax = 0;
      double dsum = 0;
      for (int b = b0; b < b0 + n[r]; ++b) {
        smin = std::min(smin, v[2 * b]);
        smax = std::max(smax, v[2 * b]);
        emax = std::max(emax, v[2 * b + 1]);
        dsum += v[2 * b + 1] - v[2 * b];
      }
      fprintf(fp, " %s[n=%d start=%.1f..%.1f end=%.1f mean=%.1f]", names[r], n[r], (smin - t0) * 0.01,
              (smax - t0) * 0.01, (emax - t0) * 0.01, dsum / n[r] * 0.01);
      if (r == 0 && t.o_grid > 0) {  // occupancy: end-time spread across frames and within them
        double fmin = 1e30, fmax = 0, wmax = 0;
        const int nfr = n[r] / t.o_grid;
        std::vector<long long> lo(nfr, LLONG_MAX), hi(nfr, 0);
        for (int b = 0; b < n[r]; ++b) {  // the device's block -> frame map (role_frame)
          const int f = (t.xcd & 1) ? (b & 7) + 8 * ((b >> 3) / t.o_grid) : b / t.o_grid;
          lo[f] = std::min(lo[f], v[2 * (b0 + b) + 1]);
          hi[f] = std::max(hi[f], v[2 * (b0 + b) + 1]);
        }
        for (int f = 0; f < nfr; ++f) {
          fmin = std::min(fmin, (hi[f] - t0) * 0.01);
          fmax = std::max(fmax, (hi[f] - t0) * 0.01);
          wmax = std::max(wmax, (hi[f] - lo[f]) * 0.01);
        }
        fprintf(fp, " occ_frame_end[%.1f..%.1f within<=%.1f]", fmin, fmax, wmax);
        std::vector<double> ends;  // workgroup end times: the balance of the stream
        for (int b = b0; b < b0 + n[r]; ++b) ends.push_back((v[2 * b + 1] - t0) * 0.01);
        std::sort(ends.begin(), ends.end());
        fprintf(fp, " occ_end_p10/50/90[%.1f %.1f %.1f]", ends[ends.size() / 10], ends[ends.size() / 2],
                ends[ends.size() * 9 / 10]);
      }
    }
    b0 += n[r];
  }
  fprintf(fp, "\n");
  fclose(fp);
}

int env_int(const char* name, int dflt) {
  const char* v = diag_env(name);
  return v && *v ? atoi(v) : dflt;
}

}  // namespace

bool tick_ok(const C3Launch& l) {
  const C3Args c = build_c3_args(l);
  return c.bits && c.ax && !l.atomic && l.prof == nullptr && l.debug == 0;
}

hipError_t launch_tick(const TickParts& p, hipStream_t s) {
  TickArgs t{};
  size_t lds = 16;
  // dispatch order: occupancy first (it streams for the whole tick from the first cycle),
  // then scoring, tile and compress+gate in the remaining workgroup slots.
  // C3H_TICK_ORDER="0312" etc. (diagnostics) lists role ids first-dispatched first.
#ifndef C3H_TICK_ORDER_DEFAULT
#define C3H_TICK_ORDER_DEFAULT 0x2130
#endif
  // (without an occupancy role -- points-in batches, drain ticks -- the chains keep the
  // tile-first order: 128^3 points-in frames 1 % faster, profiles/r3/tick_order/)
  t.order = p.occ ? C3H_TICK_ORDER_DEFAULT : 0x3210;
  if (const char* o = diag_env("C3H_TICK_ORDER"))
    if (strlen(o) == 4) {
      t.order = 0;
      for (int i = 0; i < 4; ++i) t.order |= (o[i] - '0') << (4 * i);
    }
  if (p.score) {
    const SparseSearch& a = *p.score;
    t.sq = a;
    t.s_gx = (int)std::max<int64_t>(1, std::min<int64_t>(sparse_score_blocks(a), env_int("C3H_TICK_SCORE", 16)));
    t.s_groups = (a.M + a.mpg - 1) / a.mpg;
    // one workgroup per list chunk running every model group over one box-sum pass (the
    // gathers were repeated per group): the projections then alias the basis window, which
    // must hold them
#ifndef C3H_TICK_GROUP_LOOP
#define C3H_TICK_GROUP_LOOP 1
#endif
    if (C3H_TICK_GROUP_LOOP && t.s_groups > 1 && a.D * kOC >= kFP * (kOC + 1)) {
      t.sq.group_loop = 1;
      t.s_groups = 1;
    }
    lds = std::max(lds, score_list_lds_bytes(a.D, a.mpg));
    t.n_score = t.s_gx * t.s_groups * a.nframes;
  }
  if (p.gate) {
    const SparseSearch& a = *p.gate;
    const SparseCompress& sc = *p.comp;
    t.gq = a;
    t.cr = CompressRows{sc.feat, sc.PT, sc.fmax, sc.G, sc.rows, sc.nrows, sc.F, sc.D, sc.Dpad,
                        sc.fmax_len, sc.s_feat, sc.s_G, sc.s_rows, sc.s_nrows};
    t.g_ngate = (int)((a.pstart[a.nmodes] + kBlock - 1) / kBlock);
    // the compress role on the matrix cores (round 6): 64-row blocks, D <= 128
#ifndef C3H_TICK_COMP_MFMA
#define C3H_TICK_COMP_MFMA 1
#endif
    t.comp_mfma = env_int("C3H_TICK_COMP_MFMA", C3H_TICK_COMP_MFMA) && sc.Dpad <= 128 ? 1 : 0;
    if (t.comp_mfma) {
      t.g_ncomp = (int)std::max<int64_t>(1, std::min<int64_t>((sc.H + kCR - 1) / kCR, env_int("C3H_TICK_COMP", 16)));
      lds = std::max(lds, kTLds);
    } else {
      t.g_ncomp = (int)std::max<int64_t>(1, std::min<int64_t>((sc.H + kRR - 1) / kRR, env_int("C3H_TICK_COMP", 32)));
      lds = std::max(lds, compress_rows_lds_bytes(sc.Dpad));
    }
    t.n_cg = (t.g_ngate + t.g_ncomp) * a.nframes;
  }
  if (p.tile) {
    const C3Args c = build_c3_args(*p.tile);
    t.ka = c.ka;
    // persistent tile workgroups per frame: the zero role + the work role
    const int work = std::max(1, std::min(c.tgrid - c.ka.zblocks, env_int("C3H_TICK_TILE", 48)));
    t.ka.zblocks = std::min(c.ka.zblocks, env_int("C3H_TICK_ZERO", 8));
    t.t_grid = t.ka.zblocks + work;
    t.n_tile = t.t_grid * c.nframes;
    lds = std::max(lds, c.tile_lds);
  }
  if (p.occ) {
    const C3Args c = build_c3_args(*p.occ);
    t.oa = c.oa;
    // ~256 streaming workgroups per tick whatever the batch (one per CU): the latency-bound
    // roles then see a short HBM queue and the whole tick is shortest
    // (profiles/r1/v1_occ_variants.log, v8/v9: at 32 frames per tick 12.8 us/frame with 256,
    // 14.3 with 384, 15.5 with 192)
    t.o_grid = std::max(1, std::min(c.g1, env_int("C3H_TICK_OCC", std::max(1, 256 / std::max(1, c.nframes)))));
    t.n_occ = t.o_grid * c.nframes;
    lds = std::max(lds, c.occ_lds);
    // tail stealing: the last 1/kStealDiv of every frame's chunks go to a pool shared by the
    // launch's streaming workgroups, in units of kStealUnit chunks (row-wave path only)
#ifndef C3H_TICK_STEAL_DIV
#define C3H_TICK_STEAL_DIV 16
#endif
#ifndef C3H_TICK_STEAL_UNIT
#define C3H_TICK_STEAL_UNIT 8
#endif
    const int64_t n4 = (int64_t)c.oa.gx * c.oa.gy * c.oa.gz / 4;
    const int64_t nch = (n4 + (int64_t)kBlock * kOccBitsUnroll - 1) / ((int64_t)kBlock * kOccBitsUnroll);
    const bool rowwave = c.ax && (c.oa.gx & 255) == 0 && 1024 % c.oa.gx == 0;
    const int div = env_int("C3H_TICK_STEAL_DIV", C3H_TICK_STEAL_DIV);
    const int unit = env_int("C3H_TICK_STEAL_UNIT", C3H_TICK_STEAL_UNIT);
    if (rowwave && div > 0 && unit > 0 && nch >= 2 * div) {
      const int64_t tail = nch / div;
      t.oa.steal_from = (int)(nch - tail);
      t.oa.steal_unit = unit;
      t.oa.steal_units = (int)(c.nframes * ((tail + unit - 1) / unit));
      t.oa.nframes = c.nframes;
      t.oa.steal_wgs = t.n_occ;
    }
  }
  if (const char* m = diag_env("C3H_TICK_ROLES")) {  // diagnostics only: bit mask of roles run
    const int mask = atoi(m);                       // 1 score, 2 compress+gate, 4 tile, 8 occupancy
    if (!(mask & 1)) t.n_score = 0;
    if (!(mask & 2)) t.n_cg = 0;
    if (!(mask & 4)) t.n_tile = 0;
    if (!(mask & 8)) t.n_occ = 0;
  }
  const int total = t.n_score + t.n_cg + t.n_tile + t.n_occ;
  if (total == 0) return hipSuccess;
  // XCD placement per role: its frame count a multiple of 8 and its first block at a
  // multiple of 8 in the launch
#ifndef C3H_TICK_XCD
#define C3H_TICK_XCD 15
#endif
  t.xcd = 0;
  {
    const int nb[4] = {t.n_occ, t.n_tile, t.n_cg, t.n_score};
    const int per[4] = {t.o_grid, t.t_grid, t.g_ngate + t.g_ncomp, t.s_gx * t.s_groups};
    int base = 0;  // the role's first block in the launch (dispatch order)
    for (int i = 0; i < 4; ++i) {
      const int r = (t.order >> (4 * i)) & 15;
      if (nb[r] > 0 && per[r] > 0 && base % 8 == 0 && (nb[r] / per[r]) % 8 == 0) t.xcd |= 1 << r;
      base += nb[r];
    }
    t.xcd &= C3H_TICK_XCD;
  }
  if (diag_env("C3H_TICK_PROF") && p.prof) {  // diagnostics builds only; synchronises
    DevBuf<long long>& b = *p.prof;
    if (b.n < (size_t)2 * total) {
      if (b.p) (void)hipFree(b.p);
      b.p = nullptr;
      b.n = 0;
      if (hipMalloc(&b.p, (size_t)2 * total * 8) != hipSuccess) return hipErrorOutOfMemory;
      b.n = (size_t)2 * total;
    }
    t.prof = b.p;
  }
  c3h_tick_kernel<<<(unsigned)total, kBlock, lds, s>>>(t);
  if (t.prof) tick_prof_dump(t, t.prof, total, s);
  return hipGetLastError();
}

}  // namespace c3h

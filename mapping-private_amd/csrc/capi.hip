// capi.hip -- C-ABI of libc3hlac_mi355x.so (see include/c3hlac_mi355x.h).
//
// Host-side sequencing of the voxeliser, C3-HLAC and search kernels, with the
// reference's argument semantics: setVoxelFilter's float subdivision arithmetic
// (c3_hlac/src/c3_hlac.cpp:204-231), the search mode schedule (search.cpp:384-427),
// setSceneAxis whitening (search.cpp:701-712), setRank/cleanMax list state
// (search.cpp:130-143, 683-732) and removeOverlap (search.cpp:972-992).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "c3h_internal.h"

using c3h::DevBuf;

namespace {

int fail(c3h_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}
int hip_fail(c3h_ctx* ctx, const char* what, hipError_t e) {
  return fail(ctx, C3H_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(expr)                                     \
  do {                                                   \
    hipError_t e_ = (expr);                              \
    if (e_ != hipSuccess) return hip_fail(ctx, #expr, e_); \
  } while (0)

template <class T>
int ensure(c3h_ctx* ctx, DevBuf<T>& b, size_t n) {
  if (n == 0) n = 1;
  if (b.n >= n) return C3H_OK;
  if (b.p) {
    hipError_t e = hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    if (e != hipSuccess) return hip_fail(ctx, "hipFree", e);
  }
  hipError_t e = hipMalloc(&b.p, n * sizeof(T));
  if (e != hipSuccess) {
    b.p = nullptr;
    return fail(ctx, C3H_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  b.n = n;
  return C3H_OK;
}

template <class T>
void release(DevBuf<T>& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
}

int pipe_quiesce(c3h_ctx* ctx);  // defined with the pipeline below
int pipe_flush(c3h_ctx* ctx);

// entry points that touch a context's buffers first drain its open frame stream
#define QUIESCE(ctx)                            \
  do {                                          \
    int rq_ = pipe_quiesce(ctx);                \
    if (rq_ != C3H_OK) return rq_;              \
  } while (0)

#define ENSURE(buf, n)                          \
  do {                                          \
    int rc_ = ensure(ctx, buf, (size_t)(n));    \
    if (rc_ != C3H_OK) return rc_;              \
  } while (0)

// ---- timing ------------------------------------------------------------------------
struct Timed {
  c3h_ctx* ctx;
  c3h::Timer* T;
  int slot, weight;
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  hipStream_t st;
  Timed(c3h_ctx* c, int s, int w = 1, hipStream_t on = nullptr)
      : ctx(c), T(c->parent ? &c->parent->timer : &c->timer), slot(s), weight(w), st(on ? on : c->stream) {
    if (!(T->mask >> (s + 1) & 1) || c->capture) return;
    std::lock_guard<std::mutex> g(T->mu);
    if (T->pool.empty()) {
      hipEvent_t a, b;
      if (hipEventCreate(&a) != hipSuccess) return;
      if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        return;
      }
      T->pool.push_back({a, b});
    }
    ev = T->pool.back();
    T->pool.pop_back();
    (void)hipEventRecord(ev.first, st);  // on the stream the kernels run on
  }
  ~Timed() {
    if (!ev.first) return;
    (void)hipEventRecord(ev.second, st);
    std::lock_guard<std::mutex> g(T->mu);
    T->pending[slot].push_back(c3h::TimedPair{ev.first, ev.second, weight});
  }
};

// setColor as a 256-entry table of packed (r | r_ << 8) channel pairs, one table per
// C3H_COLOR_* mode (color_chlac.hpp:148-179)
void host_lut(int color_mode, uint32_t* out) {
  const float angle_norm = M_PI / 510;  // color_chlac/include/color_chlac/color_chlac.h:9
  for (int v = 0; v < 256; ++v) {
    const float a = v * angle_norm;
    int s, c;
    if (color_mode == C3H_COLOR_CHLAC) {  // ColorCHLAC: r_ = 255 - r
      s = v;
      c = 255 - v;
    } else if (color_mode == C3H_COLOR_C3_DOUBLE) {
      s = (int)(255 * std::sin((double)a));
      c = (int)(255 * std::cos((double)a));
    } else {
      s = (int)(255 * sinf(a));
      c = (int)(255 * cosf(a));
    }
    out[v] = (uint32_t)s | ((uint32_t)c << 8);
  }
}

// search.cpp:218-251
void get_range(int mode, int r1, int r2, int r3, int* xr, int* yr, int* zr) {
  switch (mode) {
    case C3H_S_MODE_1: *xr = r1; *yr = r2; *zr = r3; break;
    case C3H_S_MODE_2: *xr = r1; *yr = r3; *zr = r2; break;
    case C3H_S_MODE_3: *xr = r2; *yr = r1; *zr = r3; break;
    case C3H_S_MODE_4: *xr = r2; *yr = r3; *zr = r1; break;
    case C3H_S_MODE_5: *xr = r3; *yr = r1; *zr = r2; break;
    default: *xr = r3; *yr = r2; *zr = r1; break;
  }
}

// search.cpp:384-427
int mode_schedule(int r1, int r2, int r3, int rotate, int* modes) {
  if (!rotate) {
    modes[0] = C3H_S_MODE_1;
    return 1;
  }
  if (r1 == r2) {
    if (r2 == r3) {
      modes[0] = C3H_S_MODE_1;
      return 1;
    }
    modes[0] = C3H_S_MODE_1; modes[1] = C3H_S_MODE_2; modes[2] = C3H_S_MODE_5;
    return 3;
  }
  if (r2 == r3) {
    modes[0] = C3H_S_MODE_1; modes[1] = C3H_S_MODE_5; modes[2] = C3H_S_MODE_6;
    return 3;
  }
  if (r1 == r3) {
    modes[0] = C3H_S_MODE_1; modes[1] = C3H_S_MODE_5; modes[2] = C3H_S_MODE_3;
    return 3;
  }
  for (int i = 0; i < 6; ++i) modes[i] = i;
  return 6;
}

// checkOverlap of SearchObjMulti (search.cpp:862-891) on host lists
int check_overlap(const c3h_det* L, int rank, int r1, int r2, int r3, int x, int y, int z,
                  int mode) {
  int xr, yr, zr, num;
  get_range(mode, r1, r2, r3, &xr, &yr, &zr);
  for (num = 0; num < rank - 1; num++) {
    int oxr, oyr, ozr;
    get_range(L[num].mode, r1, r2, r3, &oxr, &oyr, &ozr);
    int v1 = L[num].x - x;
    v1 = v1 < 0 ? -v1 - oxr : v1 - xr;
    int v2 = L[num].y - y;
    v2 = v2 < 0 ? -v2 - oyr : v2 - yr;
    int v3 = L[num].z - z;
    v3 = v3 < 0 ? -v3 - ozr : v3 - zr;
    if (v1 <= 0 && v2 <= 0 && v3 <= 0) return num;
  }
  return num;
}

struct Segs {
  std::vector<int32_t> start, len, sub;
};

// one axis of the tile decomposition.  mode1: the whole grid is one subdivision
// (hist_num == 1: c3_hlac.cpp:258,350 ignore offsets); otherwise centre voxel t >= 0
// (grid coordinate off + t) belongs to subdivision floor(t * inv_s) -- the reference's
// float arithmetic, so irregular runs caused by float rounding are reproduced.
Segs axis_segments(int div, int off, float inv_s, bool mode1, int sb, bool* covered,
                   bool* split) {
  Segs s;
  std::vector<int> runs_per_sub(std::max(sb, 1), 0);
  auto push = [&](int a0, int len, int sub) {
    for (int p = 0; p < len; p += c3h::kTileMax) {
      s.start.push_back(a0 + p);
      s.len.push_back(std::min(c3h::kTileMax, len - p));
      s.sub.push_back(sub);
      if (sub >= 0 && sub < (int)runs_per_sub.size()) runs_per_sub[sub]++;
    }
  };
  if (mode1) {
    if (div > 0) push(0, div, 0);
  } else {
    int t0 = 0;
    while (t0 < div - off) {
      const int sub = (int)floorf((float)t0 * inv_s);
      int t1 = t0 + 1;
      while (t1 < div - off && (int)floorf((float)t1 * inv_s) == sub) ++t1;
      push(off + t0, t1 - t0, sub);
      t0 = t1;
    }
  }
  *covered = true;
  *split = false;
  for (int v : runs_per_sub) {
    if (v == 0) *covered = false;
    if (v > 1) *split = true;
  }
  return s;
}

// diagnostics (env C3H_PROF=<file>): per-block phase timestamps of the tile / score
// kernels; after each instrumented launch one line per kernel is appended to the file:
// for each probe k, median over blocks of (t_k - t_0) and max over blocks of
// (t_k - min_b t_0), in microseconds (wall_clock64: 100 MHz).  Synchronises: never on.
const char* prof_path() {
  static const char* p = c3h::diag_env("C3H_PROF");
  return p && *p ? p : nullptr;
}

int prof_prepare(c3h_ctx* ctx, int64_t nblocks, long long** out) {
  *out = nullptr;
  if (!prof_path()) return C3H_OK;
  ENSURE(ctx->prof, (size_t)nblocks * 8);
  HIPCHK(hipMemsetAsync(ctx->prof.p, 0, (size_t)nblocks * 8 * 8, ctx->stream));
  *out = ctx->prof.p;
  return C3H_OK;
}

int prof_dump(c3h_ctx* ctx, const char* name, int64_t nblocks) {
  if (!prof_path()) return C3H_OK;
  std::vector<long long> t((size_t)nblocks * 8);
  HIPCHK(hipMemcpyAsync(t.data(), ctx->prof.p, t.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  long long t0min = LLONG_MAX;
  int64_t nb = 0;
  for (int64_t b = 0; b < nblocks; ++b)
    if (t[b * 8]) {
      t0min = std::min(t0min, t[b * 8]);
      ++nb;
    }
  FILE* f = fopen(prof_path(), "a");
  if (!f) return C3H_OK;
  fprintf(f, "%s blocks=%lld started=%lld", name, (long long)nblocks, (long long)nb);
  for (int k = 1; k < 8; ++k) {
    std::vector<double> d;
    double mx = 0;
    for (int64_t b = 0; b < nblocks; ++b)
      if (t[b * 8] && t[b * 8 + k]) {
        d.push_back((t[b * 8 + k] - t[b * 8]) * 0.01);
        mx = std::max(mx, (t[b * 8 + k] - t0min) * 0.01);
      }
    if (d.empty()) continue;
    std::nth_element(d.begin(), d.begin() + d.size() / 2, d.end());
    fprintf(f, " p%d[n=%zu med=%.2f max=%.2f]", k, d.size(), d[d.size() / 2], mx);
  }
  long long s0 = LLONG_MAX;  // start spread
  long long s1 = 0;
  for (int64_t b = 0; b < nblocks; ++b)
    if (t[b * 8]) {
      s0 = std::min(s0, t[b * 8]);
      s1 = std::max(s1, t[b * 8]);
    }
  fprintf(f, " start_spread=%.2f\n", nb ? (s1 - s0) * 0.01 : 0.0);
  fclose(f);
  return C3H_OK;
}

int upload_lists(c3h_ctx* ctx) {
  auto& L = ctx->lists;
  const size_t n = (size_t)L.M * L.rank;
  ENSURE(ctx->d_lists, n);
  ctx->h_lists.resize(n);
  for (size_t i = 0; i < n; ++i)
    ctx->h_lists[i] = c3h_det{L.score[i], L.x[i], L.y[i], L.z[i], L.mode[i]};
  HIPCHK(hipMemcpyAsync(ctx->d_lists.p, ctx->h_lists.data(), n * sizeof(c3h_det),
                        hipMemcpyHostToDevice, ctx->stream));
  ctx->lists_dev_valid = true;
  return C3H_OK;
}

int download_lists(c3h_ctx* ctx) {
  auto& L = ctx->lists;
  const size_t n = (size_t)L.M * L.rank;
  // through pinned memory: a pageable read-back blocks in the copy and the stream is then
  // synchronised a second time (the per-callback loop reads the lists every frame)
  if (ctx->h_dl_n < n) {
    if (ctx->h_dl) HIPCHK(hipHostFree(ctx->h_dl));
    ctx->h_dl = nullptr;
    ctx->h_dl_n = 0;
    void* hp = nullptr;
    HIPCHK(hipHostMalloc(&hp, std::max<size_t>(n, 1) * sizeof(c3h_det)));
    ctx->h_dl = static_cast<c3h_det*>(hp);
    ctx->h_dl_n = std::max<size_t>(n, 1);
  }
  HIPCHK(hipMemcpyAsync(ctx->h_dl, ctx->d_lists.p, n * sizeof(c3h_det), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  for (size_t i = 0; i < n; ++i) {
    L.score[i] = ctx->h_dl[i].score;
    L.x[i] = ctx->h_dl[i].x;
    L.y[i] = ctx->h_dl[i].y;
    L.z[i] = ctx->h_dl[i].z;
    L.mode[i] = ctx->h_dl[i].mode;
  }
  ctx->lists_host_valid = true;
  return C3H_OK;
}

void init_lists(c3h_ctx* ctx) {  // setRank: dot = 0, modes S_MODE_1 (never-initialised there)
  auto& L = ctx->lists;
  L.M = std::max(ctx->M, 1);
  L.rank = ctx->rank;
  const size_t n = (size_t)L.M * L.rank;
  L.score.assign(n, 0.0);
  L.x.assign(n, 0);
  L.y.assign(n, 0);
  L.z.assign(n, 0);
  L.mode.assign(n, C3H_S_MODE_1);
  ctx->lists_host_valid = true;
  ctx->lists_dev_valid = false;
  ctx->pending_clean = false;
}

int sync_host_lists(c3h_ctx* ctx) {
  if (!ctx->lists_host_valid) {
    int rc = download_lists(ctx);
    if (rc != C3H_OK) return rc;
  }
  if (ctx->pending_clean) {  // a cleanMax recorded while the device copy was current
    auto& L = ctx->lists;
    std::fill(L.score.begin(), L.score.end(), 0.0);
    std::fill(L.x.begin(), L.x.end(), 0);
    std::fill(L.y.begin(), L.y.end(), 0);
    std::fill(L.z.begin(), L.z.end(), 0);
    ctx->pending_clean = false;
    ctx->lists_dev_valid = false;
  }
  return C3H_OK;
}

// setData + searchPart for every scheduled mode; leaves the lists valid on the device
// setData + search for the nf frames of the last extract_frames (frame f's results at
// f * stride; d_out + f * M * rank).  clean: 0 = continue from the lists, 1 = cleanMax
// first, 2 = reset the lists as setRank does (batched frames start fresh).
// gate: -1 fill only for positions not already gated out (0: every gated-out position)
#ifndef C3H_SPARSE_SCORES
#define C3H_SPARSE_SCORES 1
#endif
constexpr int kSparseScores = C3H_SPARSE_SCORES;

// The f32 feature rows of the last extract when it wrote them as f16 (fp16 search precision
// on a large dense grid): converted on the device if the MFMA body set the flag.
int feat_rows_f32(c3h_ctx* ctx) {
  if (!ctx->feat16_pending) return C3H_OK;
  HIPCHK(c3h::launch_feat16_to_f32(ctx->feat16.p, ctx->feat16_s, ctx->feat16_flag.p, ctx->hist_num, ctx->feat_dim,
                                   ctx->feat.p, ctx->stream));
  ctx->feat16_pending = false;
  return C3H_OK;
}

int search_frames(c3h_ctx* ctx, int nf, const int32_t range[3], int32_t thr, int32_t rotate,
                  c3h_det* const* d_outs, int clean) {
  if (!ctx->have_feat) return fail(ctx, C3H_ERR_STATE, "c3h_search: no features (call c3h_extract)");
  if (!ctx->have_setup) return fail(ctx, C3H_ERR_STATE, "c3h_search: no axes (call c3h_search_setup)");
  if (!range || range[0] < 1 || range[1] < 1 || range[2] < 1)
    return fail(ctx, C3H_ERR_ARG, "c3h_search: ranges must be >= 1");
  if (ctx->feat_dim != ctx->F)
    return fail(ctx, C3H_ERR_ARG, "c3h_search: feature dimension differs from the scene axis");
  if (nf != ctx->nframes_feat) return fail(ctx, C3H_ERR_STATE, "search: frame count differs from the extract");
  const int xn = ctx->subdiv_b[0], yn = ctx->subdiv_b[1], zn = ctx->subdiv_b[2];
  const int64_t H = (int64_t)xn * yn * zn;
  if (ctx->lists.M != std::max(ctx->M, 1) || ctx->lists.rank != ctx->rank) init_lists(ctx);
  if (H < 1 || H != ctx->hist_num) return 0;  // setData returns early; search is skipped
  // projection engine (c3h_set_score_engine): the VALU list kernel (r <= 64), the matrix
  // cores over precomputed box sums (single frames), or the generic kernel (r > 64, VALU)
  const bool valu_fast = c3h::score_fast_ok(ctx->D, ctx->r);
  const bool mf = nf == 1 && !ctx->capture && c3h::score_mfma_ok(ctx->D) &&
                  (ctx->score_engine == 2 ||
                   (ctx->score_engine == 0 && (!valu_fast || H >= c3h::kBoxsumRows)));
  const bool fast = valu_fast || mf;  // the sparse (gate list) search
  if (nf > 1 && !fast) return fail(ctx, C3H_ERR_STATE, "search: batched frames need the fast path");
  int modes[6];
  const int nm = mode_schedule(range[0], range[1], range[2], rotate, modes);
  c3h::ReplayModes rm{};
  int64_t total = 0;
  for (int i = 0; i < nm; ++i) {
    int xr, yr, zr;
    get_range(modes[i], range[0], range[1], range[2], &xr, &yr, &zr);
    const int xe = xn - xr + 1, ye = yn - yr + 1, ze = zn - zr + 1;
    if (!(xe > 0 && ye > 0 && ze > 0)) continue;
    rm.m[rm.n] = c3h::ReplayMode{total, (int64_t)xe * ye * ze, xe, ye, modes[i]};
    total += rm.m[rm.n].P * ctx->M;
    rm.n++;
  }
  ENSURE(ctx->scores, (size_t)nf * std::max<int64_t>(total, 1));
  ctx->scores_n = total;
  std::vector<int64_t> layout{(int64_t)(intptr_t)ctx->scores.p, nf, ctx->M, rm.n};
  for (int i = 0; i < rm.n; ++i) {
    layout.push_back(rm.m[i].offset);
    layout.push_back(rm.m[i].P);
  }
  const bool same_layout = layout == ctx->scores_layout;
  ctx->scores_layout.clear();  // recorded again once this search's gate is enqueued (below)
  ENSURE(ctx->G, (size_t)nf * H * ctx->D);
  // sparse compress: only the non-empty rows of the extract's list (the rest stay stale
  // and every consumer gates them on exist)
  int64_t npos = 0;  // positions of every mode (0: no box fits the subdivisions)
  for (int i = 0; i < rm.n; ++i) npos += rm.m[i].P;
  // (no positions: nothing of the sparse search launches, so the compress is the dense one)
  const bool sparse_g = !ctx->g_valid && fast && ctx->rows_valid && npos > 0 &&
                        c3h::compress_rows_ok(ctx->F, ctx->Dpad);
  if (ctx->capture && !sparse_g) return 0;  // not pipelinable: the caller falls back
  if (!ctx->g_valid && !sparse_g) {  // dense compress of every frame of the extract
    int rc = feat_rows_f32(ctx);
    if (rc != C3H_OK) return rc;
    Timed t(ctx, 2, nf);
    for (int f = 0; f < nf; ++f)
      HIPCHK(c3h::launch_compress(ctx->feat.p + (size_t)f * H * ctx->F, H, ctx->F, ctx->axis_pt.p, ctx->D,
                                  ctx->Dpad, ctx->fmax.p, ctx->fmax_len, ctx->G.p + (size_t)f * H * ctx->D,
                                  nullptr, nullptr, ctx->feat_sparse ? ctx->exist.p + (size_t)f * H : nullptr,
                                  ctx->stream));
    ctx->g_valid = true;
    ctx->g_sparse = false;
  }
  const size_t per_lists = (size_t)std::max(ctx->M, 1) * ctx->rank;
  if (ctx->d_lists.n < nf * per_lists) {  // grows: frame 0's copy is re-uploaded
    if (!ctx->lists_host_valid) {
      int rc = sync_host_lists(ctx);
      if (rc != C3H_OK) return rc;
    }
    ENSURE(ctx->d_lists, nf * per_lists);
    ctx->lists_dev_valid = false;
  }
  if (clean != 2 && !ctx->lists_dev_valid) {
    int rc = upload_lists(ctx);
    if (rc != C3H_OK) return rc;
  }
  if (clean == 1 || (clean == 0 && ctx->pending_clean)) clean = 1;
  // rank 1: the replay runs in the score launch's last workgroup; on large grids its serial
  // reduction over every score chunk's partials would be the critical path, so there a
  // parallel argmax over the written scores feeds the same finalize (search.cpp:464-474)
  const bool large = !ctx->capture && nf == 1 && H >= c3h::kBoxsumRows;
  const bool use_argmax = fast && ctx->rank == 1;
  std::vector<c3h::ScoreLaunch> launches;
  for (int i = 0; i < rm.n; ++i) {
    int xr, yr, zr;
    get_range(rm.m[i].mode, range[0], range[1], range[2], &xr, &yr, &zr);
    c3h::ScoreLaunch a{};
    a.G = ctx->G.p;
    a.exist = ctx->exist.p;
    a.D = ctx->D;
    a.xn = xn;
    a.yn = yn;
    a.zn = zn;
    a.xr = xr;
    a.yr = yr;
    a.zr = zr;
    a.xe = rm.m[i].xe;
    a.ye = rm.m[i].ye;
    a.ze = (int)(rm.m[i].P / ((int64_t)rm.m[i].xe * rm.m[i].ye));
    a.thr = thr;
    a.axis_q = ctx->axis_q.p;
    a.qt = ctx->qt.p;
    a.M = ctx->M;
    a.r = ctx->r;
    a.Opad = ctx->Opad;
    a.scores = ctx->scores.p + rm.m[i].offset;
    a.order_base = (int64_t)i << 40;
    launches.push_back(a);
  }
  if (fast) {  // sparse: gate every position, project the passing ones
    c3h::SparseSearch q{};
    q.G = ctx->G.p;
    q.exist = ctx->exist.p;
    q.D = ctx->D;
    q.xn = xn;
    q.yn = yn;
    q.zn = zn;
    q.thr = thr;
    q.qt = ctx->qt.p;
    q.M = ctx->M;
    q.r = ctx->r;
    q.Opad = ctx->Opad;
    q.mpg = std::max(1, 64 / ctx->r);
    q.scores = ctx->scores.p;
    q.sparse_scores = same_layout ? kSparseScores : 0;
    q.nmodes = rm.n;
    q.score_mfma = mf ? 1 : 0;
    q.skip_empty = ctx->exist_gates_rows ? 1 : 0;
    if (mf && ctx->prec16 && ctx->Kq16 > 0) {  // fp16 search precision: f16 operands
      q.qt16 = ctx->qt16.p;
      q.Kq16 = ctx->Kq16;
    }
    q.pstart[0] = 0;
    for (int i = 0; i < rm.n; ++i) {
      const auto& a = launches[i];
      q.md[i] = c3h::ModeGeom{rm.m[i].offset, rm.m[i].P, a.xe, a.ye, a.xr, a.yr, a.zr, rm.m[i].mode};
      q.pstart[i + 1] = q.pstart[i] + rm.m[i].P;
      q.order_base[i] = (int64_t)i << 40;
    }
    const int64_t ptot = q.pstart[rm.n];
    ENSURE(ctx->glist, (size_t)nf * std::max<int64_t>(ptot, 1));
    // an epoch per launched gate (its first workgroup resets the next epoch's counters): a
    // search with no positions launches nothing and keeps the epoch
    if (!ctx->gcnt.p || ctx->gcnt_frames != nf || ctx->gcnt.n < (size_t)nf * 4 ||
        (ptot > 0 && ++ctx->search_epoch == 0)) {
      // per frame: [2] list counters | [2] finished-workgroup counters
      ENSURE(ctx->gcnt, (size_t)nf * 4);
      HIPCHK(hipMemsetAsync(ctx->gcnt.p, 0, ctx->gcnt.n * 4, ctx->stream));
      ctx->search_epoch = 1;
      ctx->gcnt_frames = nf;
    }
    q.list = ctx->glist.p;
    q.cnt = ctx->gcnt.p;
    q.done = ctx->gcnt.p + 2;
    q.epoch = ctx->search_epoch;
    q.nframes = nf;
    q.s_G = H * ctx->D;
    q.s_exist = H;
    q.s_scores = std::max<int64_t>(total, 1);
    q.s_list = std::max<int64_t>(ptot, 1);
    q.s_cnt = 4;
    q.s_lists = (int64_t)per_lists;
    for (int f = 0; f < c3h::kMaxBatch; ++f) q.outs[f] = (d_outs && f < nf) ? d_outs[f] : nullptr;
    // large grids (config 5): the box sums of every position in one streaming pass
    // before the score launch (the same (dz, dy, dx) order, so the same scores)
    if (large || mf) {
      ENSURE(ctx->gbox, (size_t)std::max<int64_t>(ptot, 1) * ctx->D);
      q.gbox = ctx->gbox.p;
      q.s_gbox = ptot * ctx->D;
    }
    const int64_t nparts = c3h::sparse_score_blocks(q);
    q.s_partials = std::max<int64_t>(nparts, 1) * ctx->M;
    if (use_argmax) {  // rank 1: the replay runs in the score launch's last workgroup
      ENSURE(ctx->partials, std::max<size_t>((size_t)nf * q.s_partials, (size_t)256 * ctx->M));
      q.partials = ctx->partials.p;
      q.lists = ctx->d_lists.p;
      q.clean = clean;
    }
    c3h::SparseCompress sc{};
    if (sparse_g) {
      sc = c3h::SparseCompress{ctx->feat.p, ctx->axis_pt.p, ctx->fmax.p, ctx->G.p, ctx->rows.p,
                               ctx->tileflags.p + 2 + (ctx->tile_epoch & 1), ctx->F, ctx->D, ctx->Dpad,
                               ctx->fmax_len, H, H * ctx->F, H * ctx->D, H, ctx->tf_stride};
      if (ctx->prec16 && ctx->Fp16 > 0) {
        sc.PT16 = ctx->axis_pt16.p;
        sc.Fp16 = ctx->Fp16;
      }
      if (ctx->feat16_pending) {
        if (sc.PT16 && H >= c3h::kCompressMfmaRows && nf == 1) {  // the f16 compress reads the f16 rows
          sc.feat16 = ctx->feat16.p;
          sc.feat16_flag = ctx->feat16_flag.p;
          sc.f16s = ctx->feat16_s;
        } else {
          int rc = feat_rows_f32(ctx);
          if (rc != C3H_OK) return rc;
        }
      }
      ctx->g_valid = true;
      ctx->g_sparse = true;
    }
    if (ctx->capture) {  // pipelined c3h_run_frames: the tick kernel runs these stages
      ctx->cap_layout.swap(layout);  // recorded by pipe_tick when the gate role is enqueued
      ctx->cap_q = q;
      ctx->cap_sc = sc;
      ctx->cap_sparse_g = sparse_g;
      ctx->cap_argmax = use_argmax;
      ctx->cap_search_valid = true;
      ctx->pending_clean = false;
      ctx->lists_host_valid = false;
      ctx->lists_dev_valid = true;
      memcpy(ctx->last_range, range, sizeof(ctx->last_range));
      return nm;
    }
    if (nf == 1) {
      int rc = prof_prepare(ctx, nparts, &q.prof);
      if (rc != C3H_OK) return rc;
    }
    {
      Timed t(ctx, 3, nf);
      HIPCHK(c3h::launch_sparse_search(q, sparse_g ? &sc : nullptr, ctx->stream));
    }
    ctx->scores_layout.swap(layout);  // the gate writes every position of this layout
    if (q.prof) {
      int rc = prof_dump(ctx, "score_list_kernel", nparts);
      if (rc != C3H_OK) return rc;
    }
    if (!use_argmax) {
      Timed t(ctx, 4, nf);
      for (int f = 0; f < nf; ++f) {
        c3h::ReplayModes rmf = rm;
        for (int i = 0; i < rmf.n; ++i) rmf.m[i].offset += f * q.s_scores;
        HIPCHK(c3h::launch_replay(ctx->scores.p, rmf, ctx->M, ctx->rank, range[0], range[1], range[2], clean,
                                  ctx->d_lists.p + f * per_lists, d_outs ? d_outs[f] : nullptr,
                                  ctx->stream));
      }
    }
  } else {
    if (ctx->g_sparse)
      return fail(ctx, C3H_ERR_STATE, "c3h_search: internal: sparse G on the dense score path");
    {
      Timed t(ctx, 3);
      for (auto& a : launches) HIPCHK(c3h::launch_score(a, ctx->stream));
    }
    ctx->scores_layout.swap(layout);
    Timed t(ctx, 4);
    HIPCHK(c3h::launch_replay(ctx->scores.p, rm, ctx->M, ctx->rank, range[0], range[1], range[2], clean,
                              ctx->d_lists.p, d_outs ? d_outs[0] : nullptr, ctx->stream));
  }
  ctx->pending_clean = false;
  ctx->lists_host_valid = false;
  ctx->lists_dev_valid = true;
  ctx->last_range[0] = range[0];
  ctx->last_range[1] = range[1];
  ctx->last_range[2] = range[2];
  return nm;
}

int run_search(c3h_ctx* ctx, const int32_t range[3], int32_t thr, int32_t rotate, c3h_det* d_out) {
  return search_frames(ctx, 1, range, thr, rotate, &d_out, 0);
}

// Exact centroids of the last voxelize (voxelize.hip vox_centroid_kernel): the fp32
// sequential means in input order, and the off-cell records (read back to the host count).
int exact_centroids(c3h_ctx* ctx) {
  if (ctx->vcent_valid) return C3H_OK;
  const int64_t ns = ctx->vns;
  const c3h::VoxArgs& a = ctx->vargs;
  const int64_t np = (int64_t)a.nblk * c3h::vox_positions(1);  // segmented list positions
  ENSURE(ctx->vcounts, (size_t)np);
  ENSURE(ctx->voffs, (size_t)np);
  ENSURE(ctx->vcur, (size_t)np);
  ENSURE(ctx->tmp_u32, (size_t)c3h::scan_blocks(np));
  ENSURE(ctx->vbucket, (size_t)std::max<int64_t>(ctx->info.n_valid, 1));
  ENSURE(ctx->vcent, (size_t)np);
  ENSURE(ctx->voffcell, (size_t)std::max<int64_t>(ns, 1) * 8);
  HIPCHK(c3h::launch_vox_centroids(a, ctx->vcounts.p, ctx->voffs.p, ctx->vcur.p, ctx->tmp_u32.p,
                                   ctx->vbucket.p, ctx->vcent.p, ctx->voffcell.p, ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->h_small, ctx->vcnt.p, c3h::kVcWords * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (ctx->h_small[c3h::kVcErr] & c3h::kVcErrBad) {
    // counts that the frame's points do not fill (the bound checks skipped every such
    // access): the accumulators held foreign sums, the next call re-zeroes them
    ctx->vtor = 0;
    ctx->table_valid = false;
    return fail(ctx, C3H_ERR_HIP, "c3h_voxelize: internal: voxel counts differ from the frame's points");
  }
  ctx->n_offcell = ctx->h_small[c3h::kVcOff];
  ctx->vcent_valid = true;
  return C3H_OK;
}

}  // namespace

extern "C" {

int c3h_version(void) { return 10000; }

int c3h_create(int hip_device, c3h_ctx** out) {
  if (!out) return C3H_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return C3H_ERR_HIP;
  if (hip_device < 0 || hip_device >= ndev) return C3H_ERR_ARG;
  c3h_ctx* ctx = new c3h_ctx();
  ctx->device = hip_device;
  auto bail = [&](int rc) {
    c3h_destroy(ctx);
    return rc;
  };
  if (hipSetDevice(hip_device) != hipSuccess) return bail(C3H_ERR_HIP);
  if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess)
    return bail(C3H_ERR_HIP);
  ctx->stream = ctx->own_stream;

  if (hipHostMalloc(&ctx->h_small, 64 * sizeof(uint32_t)) != hipSuccess) return bail(C3H_ERR_HIP);
  if (ensure(ctx, ctx->scratch, 64) != C3H_OK) return bail(C3H_ERR_NOMEM);
  if (ensure(ctx, ctx->lut, 3 * 256) != C3H_OK) return bail(C3H_ERR_NOMEM);
  uint32_t lut[3 * 256];
  for (int m = 0; m < 3; ++m) host_lut(m, lut + 256 * m);  // indexed by C3H_COLOR_*
  if (hipMemcpy(ctx->lut.p, lut, sizeof(lut), hipMemcpyHostToDevice) != hipSuccess)
    return bail(C3H_ERR_HIP);
  ctx->rank = 1;
  *out = ctx;
  return C3H_OK;
}

void c3h_destroy(c3h_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)pipe_flush(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (c3h_ctx* l : ctx->lanes) c3h_destroy(l);
  for (hipEvent_t e : ctx->lane_ev) (void)hipEventDestroy(e);
  if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->pb_vstream) {
    (void)hipStreamSynchronize(ctx->pb_vstream);
    (void)hipStreamDestroy(ctx->pb_vstream);
  }
  if (ctx->pb_vox_ev) (void)hipEventDestroy(ctx->pb_vox_ev);
  if (ctx->vcopy) {
    (void)hipStreamSynchronize(ctx->vcopy);
    (void)hipStreamDestroy(ctx->vcopy);
  }
  if (ctx->vcopy_start) (void)hipEventDestroy(ctx->vcopy_start);
  for (hipEvent_t e : ctx->vcopy_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->pb_tick_ev)
    if (e) (void)hipEventDestroy(e);
  release(ctx->grid);
  release(ctx->pts);
  release(ctx->raw);
  release(ctx->dsbuf);
  release(ctx->normals);
  release(ctx->nkeys);
  release(ctx->nkeys2);
  release(ctx->nidx);
  release(ctx->nidx2);
  release(ctx->ncstart);
  release(ctx->ncend);
  release(ctx->ntmp);
  release(ctx->dsamp);
  release(ctx->rsd_radii);
  release(ctx->rsd_types);
  release(ctx->grsd_trans);
  release(ctx->grsd_feat);
  release(ctx->vosch_feat);
  release(ctx->vacc);
  release(ctx->vmg);
  release(ctx->vtpos);
  release(ctx->vlcnt);
  release(ctx->vlists);
  release(ctx->vcnt);
  release(ctx->vpart);
  release(ctx->vcounts);
  release(ctx->voffs);
  release(ctx->vcur);
  release(ctx->vbucket);
  release(ctx->vcent);
  release(ctx->voffcell);
  release(ctx->scratch);
  release(ctx->tmp_u32);
  release(ctx->tmp_i32);
  release(ctx->feat);
  release(ctx->exist);
  release(ctx->acc64);
  release(ctx->segs);
  release(ctx->axmap);
  release(ctx->tileflags);
  release(ctx->rows);
  release(ctx->work);
  release(ctx->glist);
  release(ctx->gbox);
  release(ctx->gcnt);
  release(ctx->lut);
  release(ctx->axis_pt);
  release(ctx->axis_pt16);
  release(ctx->axis_q);
  release(ctx->fmax);
  release(ctx->G);
  release(ctx->scores);
  release(ctx->qt);
  release(ctx->partials);
  release(ctx->d_lists);
  release(ctx->prof);
  release(ctx->chist);
  release(ctx->qt16);
  release(ctx->pb_grid);
  release(ctx->pb_wlist);
  release(ctx->pb_part);
  release(ctx->pb_lim);
  release(ctx->dense_flag);
  release(ctx->pb_flags);
  release(ctx->pb_bucket);
  release(ctx->pb_xcnt);
  release(ctx->pb_moved);
  release(ctx->pb_acc);
  release(ctx->pb_accM);
  release(ctx->pb_fcnt);
  release(ctx->pb_vlist);
  release(ctx->pb_stage);
  release(ctx->pb_info);
  for (int s = 0; s < C3H_NTIMERS; ++s)
    for (auto& e : ctx->timer.pending[s]) ctx->timer.pool.push_back({e.a, e.b});
  for (auto& e : ctx->timer.pool) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (ctx->h_small) (void)hipHostFree(ctx->h_small);
  if (ctx->h_recs) (void)hipHostFree(ctx->h_recs);
  if (ctx->h_dl) (void)hipHostFree(ctx->h_dl);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

int c3h_set_stream(c3h_ctx* ctx, void* hip_stream) {
  if (!ctx) return C3H_ERR_ARG;
  hipStream_t next = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
  if (next == ctx->stream) return C3H_OK;
  HIPCHK(hipSetDevice(ctx->device));
  // an open frame stream runs its remaining ticks on the old stream, and everything queued
  // there (ticks, lanes' joins, async searches) is ordered before the new stream's work
  QUIESCE(ctx);
  if (!ctx->fork_ev) HIPCHK(hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ctx->fork_ev, ctx->stream));
  HIPCHK(hipStreamWaitEvent(next, ctx->fork_ev, 0));
  ctx->stream = next;
  return C3H_OK;
}

int c3h_synchronize(c3h_ctx* ctx) {
  if (!ctx) return C3H_ERR_ARG;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

const char* c3h_last_error(const c3h_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// c3h_voxelize of host frames: chunked copy + accumulate overlap (0: one copy, then the pass)
#ifndef C3H_VOX_CHUNKED_COPY
#define C3H_VOX_CHUNKED_COPY 0  // measured round 6: the pageable chunk copies leave ~25 us gaps (0.45 -> 0.53 ms)
#endif
constexpr bool kVoxChunkedCopy = C3H_VOX_CHUNKED_COPY;
#ifndef C3H_VOX_COPY_CHUNK_BLOCKS
#define C3H_VOX_COPY_CHUNK_BLOCKS 64  // accumulate blocks (of 4,096 points) per copied chunk
#endif
constexpr int kVoxCopyChunkBlocks = C3H_VOX_COPY_CHUNK_BLOCKS;

int c3h_voxelize(c3h_ctx* ctx, const float* xyzrgb, int64_t n, int on_device, float leaf,
                 float z_limit, c3h_grid_info* info) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (n < 0 || (n > 0 && !xyzrgb) || !(leaf > 0))
    return fail(ctx, C3H_ERR_ARG, "c3h_voxelize: bad arguments");
  if (n >= (int64_t)1 << 24)
    return fail(ctx, C3H_ERR_RANGE, "c3h_voxelize: at most 16,777,215 points per call");
  HIPCHK(hipSetDevice(ctx->device));
  ctx->have_grid = false;
  ctx->have_feat = false;
  ctx->g_valid = false;
  ctx->table_valid = false;
  ctx->vcent_valid = false;
  ctx->normals_valid = false;
  ctx->rsd_n = 0;
  ctx->n_offcell = 0;
  c3h_grid_info gi{};
  gi.leaf = leaf;
  gi.inv_leaf = 1.0f / leaf;
  const float4* d_pts = nullptr;
  // host frames of >= 2 chunks go over PCIe in chunks on a copy stream, and each chunk's
  // accumulate blocks start as soon as it lands: the accumulate pass hides under the copy
  // (a 1M-point frame: 4 chunks of 64 accumulate blocks)
  const int64_t chunk_pts = (int64_t)kVoxCopyChunkBlocks * c3h::vox_positions(1);
  const bool chunked = kVoxChunkedCopy && n > 0 && !on_device && n >= 2 * chunk_pts;
  if (n > 0) {
    if (on_device) {
      d_pts = reinterpret_cast<const float4*>(xyzrgb);
    } else {
      ENSURE(ctx->pts, (size_t)n * 4);
      if (!chunked)
        HIPCHK(hipMemcpyAsync(ctx->pts.p, xyzrgb, (size_t)n * 16, hipMemcpyHostToDevice, ctx->stream));
      d_pts = reinterpret_cast<const float4*>(ctx->pts.p);
    }
  }
  // toroidal accumulators: 2^vtb cells per axis (they only grow: a frame whose extent
  // exceeds them runs again on dims that fit it, from all-zero accumulators); entry lists
  // and partial records: one segment of the block's points per block
  uint64_t pcap = 512;
  while (pcap < (uint64_t)n) pcap <<= 1;
  const int nblk = (int)c3h::vox_blocks(n);
  c3h::VoxArgs a{};
  uint32_t* hc = ctx->h_small;
  // Every exit between the first launch and a completed scatter leaves sums in the
  // accumulators that no later frame may add onto: the next call then starts
  // from freshly zeroed accumulators (vtor = 0 forces the reallocation branch's memsets)
  struct AccGuard {
    c3h_ctx* c;
    bool armed;
    ~AccGuard() {
      if (armed) c->vtor = 0;
    }
  } acc_guard{ctx, false};
  bool wide = false;  // the extent needs more than 2^kVoxTorMaxBits accumulator cells: sorted path
  for (int attempt = 0;; ++attempt) {
    const int64_t tor = (int64_t)1 << (ctx->vtb[0] + ctx->vtb[1] + ctx->vtb[2]);
    if (ctx->vtor != tor || !ctx->vcnt.p) {  // (re)allocation: all-zero accumulators
      ctx->vtor = 0;
      ENSURE(ctx->vacc, (size_t)tor);
      ENSURE(ctx->vmg, (size_t)tor);
      ENSURE(ctx->vtpos, (size_t)tor);
      ENSURE(ctx->vcnt, c3h::kVcWords);
      HIPCHK(hipMemsetAsync(ctx->vacc.p, 0, (size_t)tor * 16, ctx->stream));
      HIPCHK(hipMemsetAsync(ctx->vmg.p, 0xff, (size_t)tor * 4, ctx->stream));
      HIPCHK(hipMemsetAsync(ctx->vcnt.p, 0, c3h::kVcWords * 4, ctx->stream));
      ctx->vtor = tor;
    }
    if (ctx->vblk_cap < nblk || !ctx->vlists.p) {  // lists: the previous frame's grid words are lost
      const int bcap = (int)std::max<int64_t>(c3h::vox_blocks((int64_t)pcap), ctx->vblk_cap);
      ENSURE(ctx->vlists, 4 * (size_t)bcap * c3h::vox_positions(1));
      ENSURE(ctx->vlcnt, (size_t)bcap * c3h::vox_positions(1));
      ENSURE(ctx->vpart, 2 * (size_t)bcap * c3h::vox_part_words());
      HIPCHK(hipMemsetAsync(ctx->vpart.p, 0, ctx->vpart.n * 4, ctx->stream));
      ctx->vlcap = (uint64_t)bcap * (uint64_t)c3h::vox_positions(1);
      ctx->vblk_cap = bcap;
      ctx->vblk_prev = 0;
      ctx->vgrid_tracked = false;
    }
    // the previous frame's grid words are cleared through its list only when its scatter
    // completed (tracked); otherwise the whole buffer is zeroed once
    const bool clear_grid = ctx->vgrid_tracked && ctx->grid.n;
    if (!ctx->vgrid_tracked && ctx->grid.n) HIPCHK(hipMemsetAsync(ctx->grid.p, 0, ctx->grid.n * 4, ctx->stream));
    ctx->vgrid_tracked = false;  // until this frame's scatter completes
    a = c3h::VoxArgs{};
    a.pts = d_pts;
    a.n = n;
    a.z_limit = z_limit;
    a.inv = gi.inv_leaf;
    a.leaf = leaf;
    a.acc = ctx->vacc.p;
    a.mg = ctx->vmg.p;
    a.tpos = ctx->vtpos.p;
    for (int ax = 0; ax < 3; ++ax) a.tb[ax] = ctx->vtb[ax];
    a.lists = ctx->vlists.p;
    a.lcap = ctx->vlcap;
    a.lcnt = ctx->vlcnt.p;
    a.part = ctx->vpart.p;
    a.nblk = nblk;
    a.nblk_prev = ctx->vblk_prev;
    a.nblk_cap = ctx->vblk_cap;
    a.cnt = ctx->vcnt.p;
    a.grid = ctx->grid.p;
    a.grid_cap = (int64_t)ctx->grid.n;
    a.par = ctx->vpar;
    a.clear_grid = clear_grid ? 1 : 0;
    acc_guard.armed = true;
    if (chunked && attempt == 0) {
      const int nch = (int)((n + chunk_pts - 1) / chunk_pts);
      if (!ctx->vcopy) HIPCHK(hipStreamCreateWithFlags(&ctx->vcopy, hipStreamNonBlocking));
      if (!ctx->vcopy_start) HIPCHK(hipEventCreateWithFlags(&ctx->vcopy_start, hipEventDisableTiming));
      while ((int)ctx->vcopy_ev.size() < nch) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->vcopy_ev.push_back(e);
      }
      // the copies overwrite ctx->pts: after everything queued that may read it
      HIPCHK(hipEventRecord(ctx->vcopy_start, ctx->stream));
      HIPCHK(hipStreamWaitEvent(ctx->vcopy, ctx->vcopy_start, 0));
      Timed t(ctx, 0);
      for (int k = 0; k < nch; ++k) {
        const int64_t off = k * chunk_pts, cnt = std::min<int64_t>(chunk_pts, n - off);
        HIPCHK(hipMemcpyAsync(ctx->pts.p + 4 * off, xyzrgb + 4 * off, (size_t)cnt * 16, hipMemcpyHostToDevice,
                              ctx->vcopy));
        HIPCHK(hipEventRecord(ctx->vcopy_ev[k], ctx->vcopy));
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->vcopy_ev[k], 0));
        c3h::VoxArgs ak = a;
        ak.blk0 = (int)(off / c3h::vox_positions(1));
        ak.clear_grid = k == 0 ? a.clear_grid : 0;
        HIPCHK(c3h::launch_vox_accum(ak, (int)c3h::vox_blocks(cnt), ctx->stream));
      }
      HIPCHK(c3h::launch_vox_scatter(a, ctx->stream));
    } else {
      int rc = prof_prepare(ctx, std::max(a.nblk, 1), &a.prof);  // diagnostics builds (C3H_PROF)
      if (rc != C3H_OK) return rc;
      {
        Timed t(ctx, 0);
        HIPCHK(c3h::launch_voxelize(a, ctx->stream));
      }
      if (a.prof) {
        rc = prof_dump(ctx, "vox_accum_kernel", std::max(a.nblk, 1));
        if (rc != C3H_OK) return rc;
        a.prof = nullptr;
      }
    }
    HIPCHK(hipMemcpyAsync(hc, ctx->vcnt.p, c3h::kVcWords * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    // the previous frame's words are cleared now (its list is spent): nothing is tracked
    // until this frame's scatter has written its own list
    ctx->vblk_prev = 0;
    if (!(hc[c3h::kVcErr] & c3h::kVcErrWrap) || (hc[c3h::kVcErr] & c3h::kVcErrRange)) break;
    // the extent exceeds the toroidal dims: dims that fit it, all-zero accumulators (the
    // wrapped sums are discarded with the old buffers), and the frame again
    int tb[3], sum = 0;
    for (int ax = 0; ax < 3; ++ax) {
      const int64_t dv = (int64_t)(int32_t)hc[c3h::kVcMax + ax] - (int32_t)hc[c3h::kVcMin + ax] + 1;
      tb[ax] = ctx->vtb[ax];
      while (((int64_t)1 << tb[ax]) < dv) ++tb[ax];
      sum += tb[ax];
    }
    if (sum > c3h::kVoxTorMaxBits) {  // a wide frame: no accumulators of that size
      wide = true;
      break;
    }
    if (attempt >= 2)  // cannot happen: the dims above fit the extent the first pass measured
      return fail(ctx, C3H_ERR_HIP, "c3h_voxelize: internal: extent still beyond the accumulators");
    for (int ax = 0; ax < 3; ++ax) ctx->vtb[ax] = tb[ax];
    ctx->vgrid_tracked = true;  // the grid holds no word of this frame (its scatter wrote none)
  }
  // from here the lists hold this frame's entries (parity a.par)
  ctx->vpar ^= 1;
  ctx->vblk_prev = nblk;
  if (hc[c3h::kVcErr] & c3h::kVcErrRange) {
    // the scatter may have stopped early (an extent beyond the dims): its sums stay behind,
    // so the next call starts from fresh accumulators
    ctx->vtor = 0;
    return fail(ctx, C3H_ERR_RANGE, "c3h_voxelize: leaf size too small (cell coordinates beyond +-2^20)");
  }
  uint64_t nvalid;
  memcpy(&nvalid, hc + c3h::kVcValid, 8);
  gi.n_valid = (int64_t)nvalid;
  if (nvalid == 0) {  // nothing scattered, and the previous frame's words are cleared
    acc_guard.armed = false;  // no point added anything
    ctx->vgrid_tracked = true;
    ctx->info = gi;
    ctx->have_grid = true;
    ctx->grid_ptr = nullptr;
    ctx->vns = 0;
    if (info) *info = gi;
    return C3H_OK;
  }
  int64_t nvox = 1;
  for (int ax = 0; ax < 3; ++ax) {
    gi.min_b[ax] = (int32_t)hc[c3h::kVcMin + ax];
    gi.max_b[ax] = (int32_t)hc[c3h::kVcMax + ax];
    gi.div_b[ax] = gi.max_b[ax] - gi.min_b[ax] + 1;
    nvox *= gi.div_b[ax];
  }
  if (nvox > 2147483647LL) {
    return fail(ctx, C3H_ERR_RANGE, "c3h_voxelize: leaf size too small for int32 voxel indices");
  }
  if (wide) {
    // the sorted path (voxelize.hip): first the accumulate pass's sums go back to zero
    // through its first-touch lists, then the frame is voxelised from its points alone
    HIPCHK(c3h::launch_vox_clear(a, ctx->stream));
    acc_guard.armed = false;
    const bool fresh = ctx->grid.n < (size_t)nvox;
    ENSURE(ctx->grid, (size_t)nvox);
    if (fresh) HIPCHK(hipMemsetAsync(ctx->grid.p, 0, ctx->grid.n * 4, ctx->stream));
    a.grid = ctx->grid.p;
    a.grid_cap = (int64_t)ctx->grid.n;
    const int64_t np = (int64_t)nblk * c3h::vox_positions(1);
    const size_t npts = (size_t)std::max<int64_t>(n, 1);
    ENSURE(ctx->vcounts, (size_t)np);
    ENSURE(ctx->vcent, (size_t)np);
    ENSURE(ctx->voffs, (size_t)np);
    ENSURE(ctx->voffcell, (size_t)std::max<uint64_t>(nvalid, 1) * 8);
    ENSURE(ctx->vbucket, npts);
    ENSURE(ctx->tmp_u32, (size_t)c3h::scan_blocks((int64_t)nvalid));
    ENSURE(ctx->nkeys, npts);
    ENSURE(ctx->nkeys2, npts);
    ENSURE(ctx->nidx, npts);
    ENSURE(ctx->nidx2, npts);
    c3h::VoxSortBufs sb{ctx->nkeys.p, ctx->nkeys2.p, ctx->nidx.p, ctx->nidx2.p, ctx->vbucket.p, ctx->tmp_u32.p,
                        reinterpret_cast<int32_t*>(ctx->voffs.p), nullptr, 0};
    int mn[3], dv[3];
    for (int ax = 0; ax < 3; ++ax) {
      mn[ax] = gi.min_b[ax];
      dv[ax] = gi.div_b[ax];
    }
    HIPCHK(c3h::launch_vox_sorted(a, mn, dv, (int64_t)nvalid, sb, ctx->vcounts.p, ctx->vcent.p, ctx->voffcell.p,
                                  ctx->stream));
    ENSURE(ctx->ntmp, std::max<size_t>(sb.tmp_bytes, 1));
    sb.tmp = ctx->ntmp.p;
    sb.tmp_bytes = ctx->ntmp.n;
    {
      Timed t(ctx, 0);
      HIPCHK(c3h::launch_vox_sorted(a, mn, dv, (int64_t)nvalid, sb, ctx->vcounts.p, ctx->vcent.p, ctx->voffcell.p,
                                    ctx->stream));
    }
    HIPCHK(hipMemcpyAsync(hc, ctx->vcnt.p, c3h::kVcWords * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->vgrid_tracked = true;
    ctx->vargs = a;
    ctx->vns = hc[c3h::kVcSlots + a.par];
    gi.n_occ = ctx->vns;
    ctx->info = gi;
    ctx->grid_ptr = ctx->grid.p;
    ctx->have_grid = true;
    ctx->table_valid = true;
    ctx->n_offcell = hc[c3h::kVcOff];
    ctx->vcent_valid = true;  // the exact centroids are in (the pass the toroidal path defers)
    if (info) *info = gi;
    return C3H_OK;
  }
  if (hc[c3h::kVcOver]) {  // the grid buffer grows (zeroed) and the scatter runs again
    ENSURE(ctx->grid, (size_t)nvox);
    HIPCHK(hipMemsetAsync(ctx->grid.p, 0, ctx->grid.n * 4, ctx->stream));
    a.grid = ctx->grid.p;
    a.grid_cap = (int64_t)ctx->grid.n;
    HIPCHK(hipMemsetAsync(ctx->vcnt.p + c3h::kVcOver, 0, 4, ctx->stream));
    {
      Timed t(ctx, 0);
      HIPCHK(c3h::launch_vox_scatter(a, ctx->stream));
    }
    HIPCHK(hipMemcpyAsync(hc, ctx->vcnt.p, c3h::kVcWords * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (hc[c3h::kVcOver]) return fail(ctx, C3H_ERR_HIP, "c3h_voxelize: internal: grid still too small");
  }
  if (hc[c3h::kVcErr] & c3h::kVcErrBad)  // (the guard re-zeroes the accumulators)
    return fail(ctx, C3H_ERR_HIP, "c3h_voxelize: internal: a listed voxel outside the frame's bounds");
  acc_guard.armed = false;  // the scatter returned every touched accumulator to zero
  ctx->vgrid_tracked = true;
  ctx->vargs = a;
  ctx->vns = hc[c3h::kVcSlots + a.par];
  gi.n_occ = ctx->vns;
  ctx->info = gi;
  ctx->grid_ptr = ctx->grid.p;
  ctx->have_grid = true;
  ctx->table_valid = true;
  if (hc[c3h::kVcFlag]) {  // centroids may leave their cells: the exact pass decides
    int rc = exact_centroids(ctx);
    if (rc != C3H_OK) return rc;
  }
  if (info) *info = gi;
  return C3H_OK;
}


int c3h_get_grid_info(c3h_ctx* ctx, c3h_grid_info* info) {
  if (!ctx || !info) return C3H_ERR_ARG;
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "no grid");
  *info = ctx->info;
  return C3H_OK;
}

int c3h_grid_device_ptr(c3h_ctx* ctx, const uint32_t** out) {
  if (!ctx || !out) return C3H_ERR_ARG;
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "no grid");
  *out = ctx->grid_ptr;
  return C3H_OK;
}

static int64_t grid_voxels(const c3h_ctx* ctx) {
  return (int64_t)ctx->info.div_b[0] * ctx->info.div_b[1] * ctx->info.div_b[2];
}

int c3h_get_grid(c3h_ctx* ctx, uint32_t* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "no grid");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t nvox = grid_voxels(ctx);
  if (nvox == 0) return C3H_OK;
  HIPCHK(hipMemcpyAsync(out, ctx->grid_ptr, (size_t)nvox * 4,
                        on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

// calc_scene_auto_threshold.cpp:92-108: one count per occupied voxel and channel
int c3h_color_histogram(c3h_ctx* ctx, int64_t* hist, int32_t accumulate) {
  if (!ctx || !hist) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "color_histogram: no grid");
  HIPCHK(hipSetDevice(ctx->device));
  ENSURE(ctx->chist, 768);
  HIPCHK(hipMemsetAsync(ctx->chist.p, 0, 768 * sizeof(unsigned long long), ctx->stream));
  HIPCHK(c3h::launch_colour_hist(ctx->grid_ptr, grid_voxels(ctx), ctx->chist.p, ctx->stream));
  unsigned long long h[768];
  HIPCHK(hipMemcpyAsync(h, ctx->chist.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < 768; ++i) hist[i] = (accumulate ? hist[i] : 0) + (int64_t)h[i];
  return C3H_OK;
}

// calc_scene_auto_threshold.cpp:111-146 (int64 where the tool's int sums would overflow,
// i.e. identical results whenever the tool's own arithmetic is defined)
int c3h_auto_threshold(const int64_t* hist, int32_t thr_out[3], double* total_ave_out) {
  if (!hist || !thr_out) return C3H_ERR_ARG;
  int64_t total = 0;
  for (int j = 0; j < 256; ++j) total += hist[j];
  if (total <= 0) return C3H_ERR_ARG;
  for (int c = 0; c < 3; ++c) {
    const int64_t* h = hist + 256 * c;
    for (int j = 0; j < 256; ++j)
      if (h[j] < 0) return C3H_ERR_ARG;
    double tot_ave = 0;  // :113-118
    for (int j = 0; j < 256; ++j) tot_ave += (double)(j * h[j]);
    tot_ave *= 1 / (double)total;
    int64_t each_num = h[0], acc = 0;  // :120-133 (eachAve[0] = 0)
    double max_var = 0;
    int thr = 0;
    for (int j = 1; j < 256; ++j) {  // :135-146, fused with the cumulative pass
      each_num += h[j];
      acc += j * h[j];
      const double each_ave = each_num == 0 ? 0.0 : (double)acc / (double)each_num;
      if (each_num != 0) {
        if (each_num == total) break;
        const double ave_sub = each_ave - tot_ave;
        const double var = ave_sub * ave_sub * (each_num / (double)(total - each_num));
        if (var > max_var) {
          max_var = var;
          thr = j;
        }
      }
    }
    thr_out[c] = thr;
    if (total_ave_out) total_ave_out[c] = tot_ave;
  }
  return C3H_OK;
}

static int compute_leaf_layout(c3h_ctx* ctx, int32_t* d_out) {
  const int64_t nvox = grid_voxels(ctx);
  const int64_t nb = c3h::leaf_layout_blocks(nvox);
  ENSURE(ctx->tmp_u32, (size_t)nb);
  HIPCHK(c3h::launch_leaf_layout(ctx->grid_ptr, nvox, d_out, ctx->tmp_u32.p, nb, ctx->stream));
  return C3H_OK;
}

int c3h_get_leaf_layout(c3h_ctx* ctx, int32_t* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "no grid");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t nvox = grid_voxels(ctx);
  if (nvox == 0) return C3H_OK;
  int32_t* dst = out;
  if (!on_device) {
    ENSURE(ctx->tmp_i32, (size_t)nvox);
    dst = ctx->tmp_i32.p;
  }
  int rc = compute_leaf_layout(ctx, dst);
  if (rc != C3H_OK) return rc;
  if (!on_device)
    HIPCHK(hipMemcpyAsync(out, dst, (size_t)nvox * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

int c3h_get_downsampled(c3h_ctx* ctx, float* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "no grid");
  if (!ctx->table_valid)
    return fail(ctx, C3H_ERR_STATE, "c3h_get_downsampled: grid was not produced by c3h_voxelize");
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t nvox = grid_voxels(ctx);
  if (nvox == 0 || ctx->info.n_occ == 0) return C3H_OK;
  int rc = exact_centroids(ctx);
  if (rc != C3H_OK) return rc;
  ENSURE(ctx->tmp_i32, (size_t)nvox);
  rc = compute_leaf_layout(ctx, ctx->tmp_i32.p);
  if (rc != C3H_OK) return rc;
  float* dst = out;
  if (!on_device) {  // not ctx->pts: it may hold the voxelize input the normals read
    ENSURE(ctx->dsbuf, (size_t)ctx->info.n_occ * 4);
    dst = ctx->dsbuf.p;
  }
  HIPCHK(c3h::launch_vox_downsampled(ctx->vargs, ctx->vcent.p, ctx->vcounts.p, ctx->tmp_i32.p, dst, ctx->stream));
  if (!on_device)
    HIPCHK(hipMemcpyAsync(out, dst, (size_t)ctx->info.n_occ * 16, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

int c3h_set_grid(c3h_ctx* ctx, const uint32_t* words, const int32_t div_b[3],
                 const int32_t min_b[3], float leaf, int on_device) {
  if (!ctx || !div_b || !min_b || !(leaf > 0)) return C3H_ERR_ARG;
  QUIESCE(ctx);
  int64_t nvox = 1;
  for (int a = 0; a < 3; ++a) {
    if (div_b[a] < 0) return fail(ctx, C3H_ERR_ARG, "c3h_set_grid: negative dims");
    nvox *= div_b[a];
  }
  if (nvox > 2147483647LL) return fail(ctx, C3H_ERR_RANGE, "c3h_set_grid: grid too large");
  if (nvox > 0 && !words) return C3H_ERR_ARG;
  HIPCHK(hipSetDevice(ctx->device));
  c3h_grid_info gi{};
  for (int a = 0; a < 3; ++a) {
    gi.div_b[a] = div_b[a];
    gi.min_b[a] = min_b[a];
    gi.max_b[a] = min_b[a] + div_b[a] - 1;
  }
  gi.leaf = leaf;
  gi.inv_leaf = 1.0f / leaf;
  gi.n_valid = -1;
  gi.n_occ = -1;
  if (on_device || nvox == 0) {
    ctx->grid_ptr = words;
  } else {
    ENSURE(ctx->grid, (size_t)nvox);
    HIPCHK(hipMemcpyAsync(ctx->grid.p, words, (size_t)nvox * 4, hipMemcpyHostToDevice, ctx->stream));
    ctx->vgrid_tracked = false;  // the next voxelize zeroes the buffer first
    ctx->grid_ptr = ctx->grid.p;
  }
  ctx->info = gi;
  ctx->have_grid = true;
  ctx->table_valid = false;
  ctx->have_feat = false;
  ctx->g_valid = false;
  return C3H_OK;
}

// C3HLAC{981,117}Estimation::setVoxelFilter + compute for nf frames of one geometry
// (grids[f], dims / min_b / leaf of ctx->info) in one set of launches; frame f's
// per-frame buffers (features, exist, tile stamps, work / row lists) sit at f * stride.
// large stand-alone extracts: the sampled density probe may skip the occupancy stream
#ifndef C3H_DENSE_PROBE
#define C3H_DENSE_PROBE 1
#endif
constexpr bool kDenseProbe = C3H_DENSE_PROBE;
// the extract after a c3h_voxelize stamps its tiles from the voxeliser's list (round 6;
// 0: stream the grid, as round 5)
#ifndef C3H_VOX_LIST_STAMP
#define C3H_VOX_LIST_STAMP 1
#endif
constexpr bool kVoxListStamp = C3H_VOX_LIST_STAMP;

static bool extract_params_ok(const c3h_extract_params* p) {
  return (p->variant == 981 || p->variant == 117) && p->color_mode >= C3H_COLOR_C3_FLOAT &&
         p->color_mode <= C3H_COLOR_CHLAC;
}

int extract_frames(c3h_ctx* ctx, const uint32_t* const* grids, int nf, const c3h_extract_params* p,
                   int32_t subdiv_out[3], int64_t* hist_num_out) {
  if (!ctx || !p) return C3H_ERR_ARG;
  if (!extract_params_ok(p))
    return fail(ctx, C3H_ERR_ARG, "c3h_extract: variant must be 981 or 117, color_mode a C3H_COLOR_* value");
  if (!ctx->have_grid) return fail(ctx, C3H_ERR_STATE, "c3h_extract: no grid");
  if (nf < 1 || nf > c3h::kMaxBatch) return fail(ctx, C3H_ERR_ARG, "extract: bad frame count");
  HIPCHK(hipSetDevice(ctx->device));
  ctx->have_feat = false;
  ctx->g_valid = false;
  ctx->rows_valid = false;
  ctx->exist_gates_rows = true;
  const int F = p->variant;
  const int* div = ctx->info.div_b;
  int32_t sb[3] = {0, 0, 0};
  int64_t hist_num = 1;
  float inv_s = 0.0f;
  auto empty = [&](const char* why) {
    ctx->err = why;
    ctx->hist_num = 0;
    ctx->feat_dim = F;
    ctx->subdiv_b[0] = sb[0];
    ctx->subdiv_b[1] = sb[1];
    ctx->subdiv_b[2] = sb[2];
    ctx->have_feat = true;
    if (subdiv_out) memcpy(subdiv_out, sb, sizeof(sb));
    if (hist_num_out) *hist_num_out = 0;
    return C3H_OK;
  };
  // setVoxelFilter (c3_hlac.cpp:204-231)
  if (p->subdiv > 0) {
    inv_s = 1.0 / p->subdiv;
    if (div[0] <= p->offset[0] || div[1] <= p->offset[1] || div[2] <= p->offset[2])
      return empty("setVoxelFilter: offset values exceed voxel grid size (empty feature)");
    for (int a = 0; a < 3; ++a) sb[a] = (int)ceilf((div[a] - p->offset[a]) * inv_s);
    hist_num = (int64_t)sb[0] * sb[1] * sb[2];
  } else if (p->subdiv < 0) {
    return empty("setVoxelFilter: invalid subdivision size (empty feature)");
  }
  // computeFeature (c3_hlac.cpp:398-401): negative thresholds -> silent empty output
  if (p->thr[0] < 0 || p->thr[1] < 0 || p->thr[2] < 0)
    return empty("computeFeature: invalid color_threshold (empty feature)");
  const bool mode1 = (hist_num == 1);
  bool covered[3], split[3];
  Segs s[3];
  for (int a = 0; a < 3; ++a)
    s[a] = axis_segments(div[a], mode1 ? 0 : p->offset[a], inv_s, mode1, mode1 ? 1 : sb[a],
                         &covered[a], &split[a]);
  const int64_t ntiles = (int64_t)s[0].start.size() * s[1].start.size() * s[2].start.size();
  for (int a = 0; a < 3; ++a)
    if (s[a].start.size() > 32767) {
      ctx->err = "c3h_extract: more than 32767 tile segments along one axis";
      return C3H_ERR_RANGE;
    }
  // voxels whose centroid leaves their cell (voxelize's exact pass) are corrected in the
  // exact 64-bit sums: the extract then runs in the atomic mode
  const bool offcell = nf == 1 && !ctx->capture && ctx->table_valid && ctx->n_offcell > 0 &&
                       ctx->grid_ptr == ctx->grid.p;
  const bool atomic = split[0] || split[1] || split[2] || offcell;
  const bool all_covered = covered[0] && covered[1] && covered[2] && ntiles > 0;
  ENSURE(ctx->feat, (size_t)nf * hist_num * F);
  ENSURE(ctx->exist, (size_t)nf * hist_num);
  ctx->nframes_feat = nf;
  ctx->feat_sparse = false;
  if (!all_covered || atomic) {
    HIPCHK(hipMemsetAsync(ctx->feat.p, 0, (size_t)nf * hist_num * F * 4, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->exist.p, 0, (size_t)nf * hist_num * 4, ctx->stream));
  }
  if (ntiles > 0) {
    int stride = 0, lmax[3] = {1, 1, 1};
    for (int a = 0; a < 3; ++a) {
      stride = std::max(stride, (int)s[a].start.size());
      for (int l : s[a].len) lmax[a] = std::max(lmax[a], l);
    }
    std::vector<int32_t> segs((size_t)3 * stride * 3, 0);
    for (int a = 0; a < 3; ++a)
      for (size_t i = 0; i < s[a].start.size(); ++i) {
        int32_t* e = &segs[((size_t)a * stride + i) * 3];
        e[0] = s[a].start[i];
        e[1] = s[a].len[i];
        e[2] = s[a].sub[i];
      }
    if (segs != ctx->h_segs || !ctx->segs.p) {  // frames of one geometry reuse the tables
      ctx->h_segs.swap(segs);
      ENSURE(ctx->segs, ctx->h_segs.size());
      HIPCHK(hipMemcpyAsync(ctx->segs.p, ctx->h_segs.data(), ctx->h_segs.size() * 4,
                            hipMemcpyHostToDevice, ctx->stream));
      // centre coordinate -> segment index per axis, for the occupancy pass
      ctx->h_axmap.assign((size_t)div[0] + div[1] + div[2], (int16_t)-1);
      int16_t* m = ctx->h_axmap.data();
      for (int a = 0; a < 3; ++a) {
        for (size_t i = 0; i < s[a].start.size(); ++i)
          for (int c = s[a].start[i]; c < s[a].start[i] + s[a].len[i]; ++c) m[c] = (int16_t)i;
        m += div[a];
      }
      ENSURE(ctx->axmap, ctx->h_axmap.size());
      HIPCHK(hipMemcpyAsync(ctx->axmap.p, ctx->h_axmap.data(), ctx->h_axmap.size() * 2,
                            hipMemcpyHostToDevice, ctx->stream));
      ++ctx->cap_h2d;
    }
    Timed t(ctx, 1, nf);  // the whole C3 stage: occupancy pass + tile kernel (+ finalize)
    // per frame: [2] reserved | [2] work-list counters | [ntiles] epoch stamps.
    // Zeroed only when (re)allocated, when the layout (stride, frame count) changes -- the
    // counters rely on every frame slot seeing every epoch -- or when the epoch wraps
    const int64_t s_tf = ntiles + 4;
    const size_t tf_n = (size_t)nf * s_tf;
    if (ctx->tileflags.n < tf_n || s_tf != ctx->tf_stride || nf != ctx->tf_frames || ++ctx->tile_epoch == 0) {
      ENSURE(ctx->tileflags, tf_n);
      HIPCHK(hipMemsetAsync(ctx->tileflags.p, 0, ctx->tileflags.n * 4, ctx->stream));
      ++ctx->cap_h2d;
      ctx->tile_epoch = 1;
      ctx->tf_stride = s_tf;
      ctx->tf_frames = nf;
    }
    if (atomic) {
      ENSURE(ctx->acc64, (size_t)nf * hist_num * 981);
      HIPCHK(hipMemsetAsync(ctx->acc64.p, 0, (size_t)nf * hist_num * 981 * 8, ctx->stream));
    }
    c3h::C3Launch l;
    for (int f = 0; f < c3h::kMaxBatch; ++f) l.grid[f] = f < nf ? grids[f] : nullptr;
    l.nframes = nf;
    l.s_feat = hist_num * F;
    l.s_h = hist_num;
    l.s_acc = hist_num * 981;
    l.s_tf = s_tf;
    l.s_work = ntiles;
    l.gx = div[0];
    l.gy = div[1];
    l.gz = div[2];
    l.segs = ctx->segs.p;
    for (int a = 0; a < 3; ++a) {
      l.nseg[a] = (int)s[a].start.size();
      l.lmax[a] = lmax[a];
      l.thr[a] = p->thr[a];
    }
    l.seg_stride = stride;
    l.sbx = mode1 ? 1 : sb[0];
    l.sby = mode1 ? 1 : sb[1];
    l.variant = F;
    l.atomic = atomic ? 1 : 0;
    l.lut = ctx->lut.p + 256 * p->color_mode;
    l.feat = ctx->feat.p;
    l.exist = ctx->exist.p;
    l.acc64 = ctx->acc64.p;
    // fp16 search precision on a large grid: the dense MFMA body writes f16 rows (the f16
    // compress reads them; every f32 reader converts them first, feat_rows_f32)
    ctx->feat16_pending = false;
    if (ctx->prec16 && nf == 1 && !ctx->capture && !atomic && F == 981 && hist_num >= c3h::kCompressMfmaRows) {
      ctx->feat16_s = (F + 7) & ~7;  // 16-B aligned rows (the compress loads 8 halves per lane)
      ENSURE(ctx->feat16, (size_t)hist_num * ctx->feat16_s);
      ENSURE(ctx->feat16_flag, 1);
      HIPCHK(hipMemsetAsync(ctx->feat16_flag.p, 0, 4, ctx->stream));
      l.feat16 = ctx->feat16.p;
      l.feat16_flag = ctx->feat16_flag.p;
      l.f16s = ctx->feat16_s;
      ctx->feat16_pending = true;
    }
    l.axmap = ctx->axmap.p;
    {  // closed-form y / z maps (uniform subdivisions from an offset): the occupancy stream
       // computes a row's segment with two scalar multiplies instead of two LDS lookups
      const int16_t* my = ctx->h_axmap.data() + div[0];
      const int16_t* mz = my + div[1];
      auto first = [](const int16_t* m, int n) {
        for (int c = 0; c < n; ++c)
          if (m[c] == 0) return c;
        return -1;
      };
      const int oy = first(my, div[1]), oz = first(mz, div[2]);
      int S = 0;
      if (oy >= 0) {
        while (oy + S < div[1] && my[oy + S] == 0) ++S;
      }
      const uint32_t magic = S > 0 ? (uint32_t)(0x100000000ull / (uint64_t)S) + 1u : 0u;
      auto closed = [&](const int16_t* m, int n, int off) {
        if (off < 0) return false;
        for (int c = 0; c < n; ++c) {
          const int v = c >= off ? (int)(((uint64_t)(uint32_t)(c - off) * magic) >> 32) : -1;
          if (v != m[c]) return false;
        }
        return true;
      };
      const bool ok = S > 0 && oz >= 0 && closed(my, div[1], oy) && closed(mz, div[2], oz);
      l.ar_s = ok ? S : 0;
      l.ar_oy = oy;
      l.ar_oz = oz;
      l.ar_magic = magic;
    }
    ENSURE(ctx->work, (size_t)nf * ntiles);
    l.tf = ctx->tileflags.p;
    l.work = ctx->work.p;
    l.rows = nullptr;
    if (!atomic) {  // the non-empty rows feed the sparse compress of the search
      ENSURE(ctx->rows, (size_t)nf * hist_num);
      l.rows = ctx->rows.p;
    }
    ctx->rows_valid = !atomic;
    l.epoch = ctx->tile_epoch;
    l.zero_empty = (!atomic && all_covered) ? 1 : 0;
    // direct mode writes only the non-empty rows' features; the rest stay stale (their
    // exist is 0, every reader gates on it) -- 8 MB (117) / 69 MB (981) less per frame
    l.zero_feat = 0;
    ctx->feat_sparse = l.zero_empty && !l.zero_feat;
    l.ntiles = ntiles;
    l.debug = 0;
    l.prof = nullptr;
    l.dense = nullptr;
    // the grid of the last c3h_voxelize: its occupied voxels are listed (vox_scatter / the
    // sorted path), so the tiles are stamped from the list instead of the 4 B/voxel stream
    // (sparse frames: 16 B of list work per occupied voxel below the grid's 4 B per voxel)
    const bool from_list = kVoxListStamp && !ctx->capture && nf == 1 && ctx->table_valid &&
                           ctx->grid_ptr == ctx->grid.p && ctx->vargs.lists &&
                           (int64_t)ctx->vns * 16 < (int64_t)div[0] * div[1] * div[2];
    if (from_list) {
      const c3h::VoxArgs& va = ctx->vargs;
      l.vl_words = va.lists + (size_t)(2 + va.par) * va.lcap;
      l.vl_counts = va.part + (size_t)va.par * va.nblk_cap * c3h::vox_part_words() + c3h::kVoxPartNew;
      l.vl_count_stride = c3h::vox_part_words();
      l.vl_seg = (int)c3h::vox_positions(1);
      l.vl_nseg = va.nblk;
    }
    if (!from_list && !ctx->capture && nf == 1 && ntiles >= 65536 && l.zero_empty && !atomic && kDenseProbe) {
      ENSURE(ctx->dense_flag, 1);
      l.dense = ctx->dense_flag.p;
    }
    if (const char* dbg = c3h::diag_env("C3H_C3_DEBUG")) l.debug = atoi(dbg);  // diagnostics only
    const int64_t tgrid = c3h::c3hlac_grid(l);
    if (nf == 1) {
      int rc = prof_prepare(ctx, tgrid, &l.prof);
      if (rc != C3H_OK) return rc;
    }
    if (ctx->capture) {  // pipelined c3h_run_frames: the tick kernel runs this launch
      ctx->cap_c3 = l;
      ctx->cap_c3_valid = true;
    } else {
      HIPCHK(c3h::launch_c3hlac(l, ctx->stream));
      if (l.prof) {
        int rc = prof_dump(ctx, "c3hlac_tile_kernel", tgrid);
        if (rc != C3H_OK) return rc;
      }
      if (offcell) {
        const int sbv[3] = {l.sbx, l.sby, mode1 ? 1 : sb[2]};
        HIPCHK(c3h::launch_offcell_delta(ctx->voffcell.p, (int)ctx->n_offcell, l, mode1 ? 1 : 0, p->offset, sbv,
                                         inv_s, ctx->stream));
      }
      if (atomic)
        HIPCHK(c3h::launch_c3_finalize(ctx->acc64.p, hist_num, F, ctx->feat.p, ctx->exist.p, nf, ctx->stream));
    }
  }
  ctx->hist_num = hist_num;
  ctx->feat_dim = F;
  ctx->subdiv_b[0] = sb[0];
  ctx->subdiv_b[1] = sb[1];
  ctx->subdiv_b[2] = sb[2];
  ctx->last = *p;
  ctx->have_feat = true;
  if (subdiv_out) memcpy(subdiv_out, sb, sizeof(sb));
  if (hist_num_out) *hist_num_out = hist_num;
  return C3H_OK;
}

int c3h_extract(c3h_ctx* ctx, const c3h_extract_params* p, int32_t subdiv_out[3],
                int64_t* hist_num_out) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  const uint32_t* g = ctx->grid_ptr;
  return extract_frames(ctx, &g, 1, p, subdiv_out, hist_num_out);
}

// sensor_msgs/PointCloud2 ingestion (pcl::fromROSMsg, detect_object.cpp:142)
static int pc2_check(c3h_ctx* ctx, uint32_t height, uint32_t width, uint32_t point_step, uint32_t row_step,
                     const int32_t off[4]) {
  if (!off) return fail(ctx, C3H_ERR_ARG, "pointcloud2: no field offsets");
  for (int k = 0; k < 4; ++k)
    if ((k < 3 && off[k] < 0) || off[k] + 4 > (int64_t)point_step)
      return fail(ctx, C3H_ERR_ARG, "pointcloud2: field x/y/z missing or outside point_step");
  if (height > 1 && (uint64_t)row_step < (uint64_t)width * point_step)
    return fail(ctx, C3H_ERR_ARG, "pointcloud2: row_step < width * point_step");
  return C3H_OK;
}

int c3h_pointcloud2_to_xyzrgb(const void* d_data, uint32_t height, uint32_t width, uint32_t point_step,
                              uint32_t row_step, const int32_t offsets[4], int32_t is_bigendian, float* d_out,
                              void* hip_stream) {
  if ((!d_data || !d_out) && (uint64_t)height * width > 0) return C3H_ERR_ARG;
  int rc = pc2_check(nullptr, height, width, point_step, row_step, offsets);
  if (rc != C3H_OK) return rc;
  return c3h::launch_pc2_convert(d_data, height, width, point_step, row_step, offsets, is_bigendian ? 1 : 0, d_out,
                                 (hipStream_t)hip_stream) == hipSuccess
             ? C3H_OK
             : C3H_ERR_HIP;
}

int c3h_voxelize_pointcloud2(c3h_ctx* ctx, const void* data, uint32_t height, uint32_t width, uint32_t point_step,
                             uint32_t row_step, const int32_t offsets[4], int32_t is_bigendian, int on_device,
                             float leaf, float z_limit, c3h_grid_info* info) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  int rc = pc2_check(ctx, height, width, point_step, row_step, offsets);
  if (rc != C3H_OK) return rc;
  const int64_t n = (int64_t)height * width;
  if (n > 0 && !data) return fail(ctx, C3H_ERR_ARG, "pointcloud2: no data");
  if (n >= (int64_t)1 << 24) return fail(ctx, C3H_ERR_RANGE, "c3h_voxelize: at most 16,777,215 points per call");
  HIPCHK(hipSetDevice(ctx->device));
  const void* src = data;
  if (n > 0 && !on_device) {  // the message bytes: rows of row_step (the last one may be short)
    const size_t bytes = (size_t)(height - 1) * (height > 1 ? row_step : 0) + (size_t)width * point_step;
    ENSURE(ctx->raw, (bytes + 3) / 4);
    HIPCHK(hipMemcpyAsync(ctx->raw.p, data, bytes, hipMemcpyHostToDevice, ctx->stream));
    src = ctx->raw.p;
  }
  ENSURE(ctx->pts, (size_t)std::max<int64_t>(n, 1) * 4);
  HIPCHK(c3h::launch_pc2_convert(src, height, width, point_step, height > 1 ? row_step : width * point_step, offsets,
                                 is_bigendian ? 1 : 0, ctx->pts.p, ctx->stream));
  return c3h_voxelize(ctx, ctx->pts.p, n, 1, leaf, z_limit, info);
}

// ---- normals, RSD, GRSD, VOSCH (rsd.hip; grsd_colorCHLAC_tools.hpp) -----------------
// radius-search grid over the points of the last c3h_voxelize (those it kept)
static int nbr_grid(c3h_ctx* ctx, float cell) {
  const c3h::VoxArgs& a = ctx->vargs;
  c3h::NbrGrid g{};
  g.pts = a.pts;
  g.n = a.n;
  g.cell = cell;
  g.inv_cell = 1.0f / cell;
  for (int ax = 0; ax < 3; ++ax) {
    const double lo = (double)ctx->info.min_b[ax] * ctx->info.leaf, hi = (double)(ctx->info.max_b[ax] + 1) * ctx->info.leaf;
    g.origin[ax] = (float)(lo - cell);
    g.dim[ax] = (int)std::ceil((hi - lo) / cell) + 3;
  }
  const int64_t ncell = (int64_t)g.dim[0] * g.dim[1] * g.dim[2];
  if (ncell > ((int64_t)1 << 27)) return fail(ctx, C3H_ERR_RANGE, "normals: more than 2^27 search cells");
  const size_t n = (size_t)std::max<int64_t>(g.n, 1);
  ENSURE(ctx->nkeys, n);
  ENSURE(ctx->nkeys2, n);
  ENSURE(ctx->nidx, n);
  ENSURE(ctx->nidx2, n);
  ENSURE(ctx->ncstart, (size_t)ncell);
  ENSURE(ctx->ncend, (size_t)ncell);
  g.cstart = ctx->ncstart.p;
  g.cend = ctx->ncend.p;
  size_t tb = 0;
  HIPCHK(c3h::nbr_build(g, ctx->nkeys.p, ctx->nkeys2.p, ctx->nidx.p, ctx->nidx2.p, nullptr, &tb, ctx->stream));
  ENSURE(ctx->ntmp, std::max<size_t>(tb, 1));
  tb = ctx->ntmp.n;
  HIPCHK(c3h::nbr_build(g, ctx->nkeys.p, ctx->nkeys2.p, ctx->nidx.p, ctx->nidx2.p, ctx->ntmp.p, &tb, ctx->stream));
  ctx->nbr = g;
  return C3H_OK;
}

int c3h_compute_normals(c3h_ctx* ctx, float radius, const float viewpoint[3]) {
  if (!ctx || !(radius > 0)) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid || !ctx->table_valid)
    return fail(ctx, C3H_ERR_STATE, "compute_normals: needs the points of a c3h_voxelize");
  HIPCHK(hipSetDevice(ctx->device));
  ctx->normals_valid = false;
  int rc = nbr_grid(ctx, radius);
  if (rc != C3H_OK) return rc;
  ENSURE(ctx->normals, (size_t)std::max<int64_t>(ctx->vargs.n, 1));
  const float vp0[3] = {0.0f, 0.0f, 0.0f};
  HIPCHK(c3h::launch_normals(ctx->nbr, radius, viewpoint ? viewpoint : vp0, ctx->normals.p, ctx->stream));
  ctx->normals_valid = true;
  return C3H_OK;
}

int c3h_get_normals(c3h_ctx* ctx, float* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->normals_valid) return fail(ctx, C3H_ERR_STATE, "get_normals: c3h_compute_normals first");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(out, ctx->normals.p, (size_t)ctx->vargs.n * 16,
                        on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

// extractGRSDSignature21 (grsd_colorCHLAC_tools.hpp:131-296) into grsd_feat (H x 20)
static int grsd_frames(c3h_ctx* ctx, const c3h_grsd_params* p, int32_t sb[3], int64_t* Hout) {
  if (!ctx->normals_valid) return fail(ctx, C3H_ERR_STATE, "extract_grsd: c3h_compute_normals first");
  const int* div = ctx->info.div_b;
  int64_t H = 1;
  float inv_s = 0.0f;
  sb[0] = sb[1] = sb[2] = 0;
  *Hout = 0;
  if (p->subdiv > 0) {
    inv_s = 1.0 / p->subdiv;
    if (div[0] <= p->offset[0] || div[1] <= p->offset[1] || div[2] <= p->offset[2]) return C3H_OK;  // :150-153
    for (int a = 0; a < 3; ++a) sb[a] = (int)ceilf((div[a] - p->offset[a]) * inv_s);
    H = (int64_t)sb[0] * sb[1] * sb[2];
  } else if (p->subdiv < 0) {
    return C3H_OK;  // :159-162: invalid subdivision size -> empty
  } else {
    sb[0] = sb[1] = sb[2] = 1;
  }
  const int64_t nc = ctx->info.n_occ;
  const int64_t nvox = grid_voxels(ctx);
  int rc = exact_centroids(ctx);
  if (rc != C3H_OK) return rc;
  ENSURE(ctx->tmp_i32, (size_t)std::max<int64_t>(nvox, 1));
  rc = compute_leaf_layout(ctx, ctx->tmp_i32.p);
  if (rc != C3H_OK) return rc;
  ENSURE(ctx->dsamp, (size_t)std::max<int64_t>(nc, 1));
  HIPCHK(c3h::launch_vox_downsampled(ctx->vargs, ctx->vcent.p, ctx->vcounts.p, ctx->tmp_i32.p,
                                     reinterpret_cast<float*>(ctx->dsamp.p), ctx->stream));
  // RSD radius: max(rsd_radius_search, voxel_size / 2 * sqrt(3)) (:172)
  const float max_dist = (float)std::max((double)p->rsd_radius, (double)ctx->info.leaf / 2 * std::sqrt(3.0));
  if (max_dist > 4 * ctx->nbr.cell) {
    // a wide RSD radius (large leaves: leaf sqrt(3)/2 > 4 x the normal radius) gets a search
    // grid of its own radius; the normals are already computed, and the RSD's per-bin
    // min/max angles do not depend on the neighbour visiting order
    rc = nbr_grid(ctx, max_dist);
    if (rc != C3H_OK) return rc;
  }
  ENSURE(ctx->rsd_radii, (size_t)std::max<int64_t>(nc, 1));
  ENSURE(ctx->rsd_types, (size_t)std::max<int64_t>(nc, 1));
  HIPCHK(c3h::launch_rsd(ctx->nbr, ctx->normals.p, ctx->dsamp.p, nc, max_dist, ctx->rsd_radii.p, ctx->rsd_types.p,
                         ctx->stream));
  ctx->rsd_n = nc;
  ENSURE(ctx->grsd_trans, (size_t)H * 36);
  HIPCHK(hipMemsetAsync(ctx->grsd_trans.p, 0, (size_t)H * 36 * 4, ctx->stream));
  c3h::GrsdArgs ga{};
  ga.cent = ctx->dsamp.p;
  ga.nc = nc;
  ga.layout = ctx->tmp_i32.p;
  ga.types = ctx->rsd_types.p;
  ga.trans = ctx->grsd_trans.p;
  for (int a = 0; a < 3; ++a) {
    ga.div_b[a] = div[a];
    ga.min_b[a] = ctx->info.min_b[a];
    ga.off[a] = p->subdiv > 0 ? p->offset[a] : 0;
    ga.sb[a] = sb[a];
  }
  ga.leaf = ctx->info.leaf;
  ga.inv_leaf = 1.0f / ctx->info.leaf;
  ga.inv_s = inv_s;
  ga.hist1 = H == 1 ? 1 : 0;
  HIPCHK(c3h::launch_grsd(ga, ctx->stream));
  ENSURE(ctx->grsd_feat, (size_t)H * 20);
  // NORMALIZE_GRSD = 20 / 26 (grsd_colorCHLAC_tools.h:32) when is_normalize
  HIPCHK(c3h::launch_grsd_feat(ctx->grsd_trans.p, H, p->normalize ? (float)(20.0 / 26) : 1.0f, ctx->grsd_feat.p, 20,
                               ctx->stream));
  *Hout = H;
  return C3H_OK;
}

int c3h_extract_grsd(c3h_ctx* ctx, const c3h_grsd_params* p, int32_t subdiv_out[3], int64_t* hist_num) {
  if (!ctx || !p) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid || !ctx->table_valid) return fail(ctx, C3H_ERR_STATE, "extract_grsd: no c3h_voxelize grid");
  HIPCHK(hipSetDevice(ctx->device));
  ctx->have_feat = false;
  ctx->g_valid = false;
  ctx->rows_valid = false;
  ctx->exist_gates_rows = false;
  int32_t sb[3];
  int64_t H = 0;
  int rc = grsd_frames(ctx, p, sb, &H);
  if (rc != C3H_OK) return rc;
  ctx->feat16_pending = false;
  ENSURE(ctx->feat, (size_t)std::max<int64_t>(H, 1) * 20);
  ENSURE(ctx->exist, (size_t)std::max<int64_t>(H, 1));
  if (H > 0) {
    HIPCHK(hipMemcpyAsync(ctx->feat.p, ctx->grsd_feat.p, (size_t)H * 20 * 4, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(c3h::launch_exist_rule(ctx->feat.p, H, 20, C3H_EXIST_GRSD, ctx->exist.p, ctx->stream));
  }
  ctx->hist_num = H;
  ctx->feat_dim = 20;
  for (int a = 0; a < 3; ++a) ctx->subdiv_b[a] = sb[a];
  ctx->nframes_feat = 1;
  ctx->feat_sparse = false;
  ctx->have_feat = true;
  if (subdiv_out) memcpy(subdiv_out, sb, sizeof(sb));
  if (hist_num) *hist_num = H;
  return C3H_OK;
}

int c3h_get_rsd(c3h_ctx* ctx, float* radii, int32_t* types, int on_device) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (ctx->rsd_n == 0 && !ctx->normals_valid) return fail(ctx, C3H_ERR_STATE, "get_rsd: no RSD computed");
  HIPCHK(hipSetDevice(ctx->device));
  const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (radii && ctx->rsd_n) HIPCHK(hipMemcpyAsync(radii, ctx->rsd_radii.p, (size_t)ctx->rsd_n * 8, k, ctx->stream));
  if (types && ctx->rsd_n) HIPCHK(hipMemcpyAsync(types, ctx->rsd_types.p, (size_t)ctx->rsd_n * 4, k, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return (int)std::min<int64_t>(ctx->rsd_n, INT_MAX);
}

// extractVOSCH (grsd_colorCHLAC_tools.hpp:832-843): [GRSD-20 | C3-HLAC-117] per subdivision
int c3h_extract_vosch(c3h_ctx* ctx, const c3h_grsd_params* p, const int32_t thr[3], int32_t color_mode,
                      int32_t subdiv_out[3], int64_t* hist_num) {
  if (!ctx || !p || !thr) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_grid || !ctx->table_valid) return fail(ctx, C3H_ERR_STATE, "extract_vosch: no c3h_voxelize grid");
  HIPCHK(hipSetDevice(ctx->device));
  int32_t sb[3];
  int64_t H = 0;
  int rc = grsd_frames(ctx, p, sb, &H);
  if (rc != C3H_OK) return rc;
  c3h_extract_params e{};
  e.variant = 117;
  for (int a = 0; a < 3; ++a) {
    e.thr[a] = thr[a];
    e.offset[a] = p->offset[a];
  }
  e.subdiv = p->subdiv;
  e.color_mode = color_mode;
  const uint32_t* g = ctx->grid_ptr;
  int32_t sb2[3];
  int64_t H2 = 0;
  rc = extract_frames(ctx, &g, 1, &e, sb2, &H2);
  if (rc != C3H_OK) return rc;
  if (H2 != H) return fail(ctx, C3H_ERR_STATE, "extract_vosch: GRSD / C3 subdivisions differ");
  ENSURE(ctx->vosch_feat, (size_t)std::max<int64_t>(H, 1) * 137);
  HIPCHK(c3h::launch_vosch_concat(ctx->grsd_feat.p, ctx->feat.p, ctx->exist.p, H, ctx->vosch_feat.p, ctx->stream));
  std::swap(ctx->feat, ctx->vosch_feat);
  ctx->feat_dim = 137;
  ctx->feat_sparse = false;
  ctx->g_valid = false;
  ctx->rows_valid = false;
  ctx->exist_gates_rows = false;
  if (subdiv_out) memcpy(subdiv_out, sb, sizeof(sb));
  if (hist_num) *hist_num = H;
  return C3H_OK;
}

// SearchObj::setData (search.cpp:539-658) with caller-computed features (VOSCH, GRSD,
// ConVOSCH, or C3-HLAC rows from elsewhere): the next search consumes them
int c3h_set_features(c3h_ctx* ctx, const float* feat, const int32_t subdiv_b[3], int32_t dim,
                     const int32_t* exist, int32_t exist_rule, int on_device) {
  if (!ctx || !subdiv_b || dim <= 0) return C3H_ERR_ARG;
  if (subdiv_b[0] < 0 || subdiv_b[1] < 0 || subdiv_b[2] < 0) return fail(ctx, C3H_ERR_ARG, "set_features: subdiv_b");
  if (!exist && (exist_rule < 0 || exist_rule > 2)) return fail(ctx, C3H_ERR_ARG, "set_features: exist rule");
  if (exist_rule == C3H_EXIST_VOSCH && dim < 22) return fail(ctx, C3H_ERR_ARG, "set_features: VOSCH rule needs dim >= 22");
  if (exist_rule == C3H_EXIST_GRSD && dim < 20) return fail(ctx, C3H_ERR_ARG, "set_features: GRSD rule needs dim >= 20");
  if (exist_rule == C3H_EXIST_C3HLAC && dim < 2) return fail(ctx, C3H_ERR_ARG, "set_features: bad dim");
  QUIESCE(ctx);
  HIPCHK(hipSetDevice(ctx->device));
  const int64_t H = (int64_t)subdiv_b[0] * subdiv_b[1] * subdiv_b[2];
  if (H > 0 && !feat) return C3H_ERR_ARG;
  ctx->feat16_pending = false;  // the caller's rows replace the extract's
  ctx->have_feat = false;
  ctx->g_valid = false;
  ctx->rows_valid = false;
  ctx->exist_gates_rows = false;
  ENSURE(ctx->feat, (size_t)H * dim);
  ENSURE(ctx->exist, (size_t)H);
  if (H > 0) {
    const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    HIPCHK(hipMemcpyAsync(ctx->feat.p, feat, (size_t)H * dim * sizeof(float), k, ctx->stream));
    if (exist)
      HIPCHK(hipMemcpyAsync(ctx->exist.p, exist, (size_t)H * sizeof(int32_t), k, ctx->stream));
    else
      HIPCHK(c3h::launch_exist_rule(ctx->feat.p, H, dim, exist_rule, ctx->exist.p, ctx->stream));
  }
  if (!on_device) HIPCHK(hipStreamSynchronize(ctx->stream));  // host arrays may be freed on return
  ctx->hist_num = H;
  ctx->feat_dim = dim;
  for (int a = 0; a < 3; ++a) ctx->subdiv_b[a] = subdiv_b[a];
  ctx->nframes_feat = 1;
  ctx->feat_sparse = false;
  ctx->have_feat = true;
  return C3H_OK;
}

// rows h with exist[h] == 0 read as 0 (buffers whose empty rows are left stale)
static int masked_readback(c3h_ctx* ctx, const float* src, int W, float* out, int on_device) {
  const size_t n = (size_t)ctx->hist_num * W;
  float* dst = out;
  c3h::DevBuf<float> tmp;
  if (!on_device) {
    int rc = ensure(ctx, tmp, n);
    if (rc != C3H_OK) return rc;
    dst = tmp.p;
  }
  hipError_t e = c3h::launch_masked_rows(src, ctx->exist.p, ctx->hist_num, W, dst, ctx->stream);
  if (e == hipSuccess && !on_device) e = hipMemcpyAsync(out, dst, n * 4, hipMemcpyDeviceToHost, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (!on_device) release(tmp);
  if (e != hipSuccess) return fail(ctx, C3H_ERR_HIP, std::string("readback: ") + hipGetErrorString(e));
  return C3H_OK;
}

int c3h_get_feature_info(c3h_ctx* ctx, int32_t subdiv_out[3], int64_t* hist_num, int32_t* dim) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  const bool h = ctx->have_feat;
  if (subdiv_out)
    for (int a = 0; a < 3; ++a) subdiv_out[a] = h ? ctx->subdiv_b[a] : 0;
  if (hist_num) *hist_num = h ? ctx->hist_num : 0;
  if (dim) *dim = h ? ctx->feat_dim : 0;
  return C3H_OK;
}

int c3h_get_features(c3h_ctx* ctx, float* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_feat) return fail(ctx, C3H_ERR_STATE, "no features");
  HIPCHK(hipSetDevice(ctx->device));
  const size_t n = (size_t)ctx->hist_num * ctx->feat_dim;
  {
    int rc = feat_rows_f32(ctx);
    if (rc != C3H_OK) return rc;
  }
  if (n && ctx->feat_sparse) return masked_readback(ctx, ctx->feat.p, ctx->feat_dim, out, on_device);
  if (n) HIPCHK(hipMemcpyAsync(out, ctx->feat.p, n * 4, on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

int c3h_get_exist(c3h_ctx* ctx, int32_t* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->have_feat) return fail(ctx, C3H_ERR_STATE, "no features");
  HIPCHK(hipSetDevice(ctx->device));
  const size_t n = (size_t)ctx->hist_num;
  if (n) HIPCHK(hipMemcpyAsync(out, ctx->exist.p, n * 4, on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

int c3h_set_search_precision(c3h_ctx* ctx, int32_t fp16) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  ctx->prec16 = fp16 != 0;
  ctx->g_valid = false;
  return C3H_OK;
}

int c3h_set_score_engine(c3h_ctx* ctx, int32_t engine) {
  if (!ctx) return C3H_ERR_ARG;
  if (engine < 0 || engine > 2) return fail(ctx, C3H_ERR_ARG, "c3h_set_score_engine: engine must be 0, 1 or 2");
  QUIESCE(ctx);
  ctx->score_engine = engine;
  return C3H_OK;
}

// the bases on the device (D a multiple of 4 when D <= 160; see c3h_search_setup)
static int search_setup_dev(c3h_ctx* ctx, const float* axis_p, const float* var, int32_t D, int32_t F,
                            const float* axis_q, int32_t M, int32_t r, const float* feature_max,
                            int32_t feature_max_len, int32_t D_user) {
  HIPCHK(hipSetDevice(ctx->device));
  // the bases are replaced with synchronous copies: queued kernels of this context may
  // still read them
  HIPCHK(hipStreamSynchronize(ctx->stream));
  const int Dpad = (D + 7) / 8 * 8;
  std::vector<float> pt((size_t)F * Dpad, 0.0f);
  for (int d = 0; d < D; ++d) {
    // setSceneAxis with whitening: row d scaled by 1/sqrt(var(d)) (search.cpp:701-712)
    const float w = var ? (float)(1 / std::sqrt((double)var[d])) : 1.0f;
    for (int j = 0; j < F; ++j) {
      float v;
      if (axis_p) v = var ? w * axis_p[(size_t)d * F + j] : axis_p[(size_t)d * F + j];
      else v = (d == j) ? 1.0f : 0.0f;
      pt[(size_t)j * Dpad + d] = v;
    }
  }
  ENSURE(ctx->axis_pt, pt.size());
  HIPCHK(hipMemcpy(ctx->axis_pt.p, pt.data(), pt.size() * 4, hipMemcpyHostToDevice));
  // f16 copy for the fp16 matrix-core compress: 128 columns x Fp16, column-major
  if (D <= 128) {
    const int Fp16 = (F + 15) / 16 * 16;
    std::vector<_Float16> p16((size_t)128 * Fp16, (_Float16)0.0f);
    for (int d = 0; d < D; ++d)
      for (int j = 0; j < F; ++j) p16[(size_t)d * Fp16 + j] = (_Float16)pt[(size_t)j * Dpad + d];
    ENSURE(ctx->axis_pt16, p16.size());
    HIPCHK(hipMemcpy(ctx->axis_pt16.p, p16.data(), p16.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    ctx->Fp16 = Fp16;
  } else {
    ctx->Fp16 = 0;
  }
  ENSURE(ctx->axis_q, (size_t)M * r * D);
  HIPCHK(hipMemcpy(ctx->axis_q.p, axis_q, (size_t)M * r * D * 4, hipMemcpyHostToDevice));
  // transposed basis for the fast score path: qt[d][m*r + i] = axis_q[m][i][d]
  // + 16 zero columns: a score workgroup's window of whole models may run past M*r
  const int Opad = (M * r + 15) / 16 * 16 + 16;
  std::vector<float> qt((size_t)D * Opad, 0.0f);
  for (int m = 0; m < M; ++m)
    for (int i = 0; i < r; ++i)
      for (int d = 0; d < D; ++d) qt[(size_t)d * Opad + m * r + i] = axis_q[((size_t)m * r + i) * D + d];
  ENSURE(ctx->qt, qt.size());
  HIPCHK(hipMemcpy(ctx->qt.p, qt.data(), qt.size() * 4, hipMemcpyHostToDevice));
  ctx->Opad = Opad;
  // f16 basis for the fp16 matrix-core projection: column-major [Opad][16 * Kq16] (a lane's
  // 8 consecutive k are one 16-B load), zero past D and past M * r
  ctx->Kq16 = 0;
  if (c3h::score_mfma_ok(D)) {
    const int Kq = (D + 15) / 16, KH = 16 * Kq;
    std::vector<_Float16> q16((size_t)Opad * KH, (_Float16)0.0f);
    for (int c = 0; c < M * r; ++c)
      for (int d = 0; d < D; ++d) q16[(size_t)c * KH + d] = (_Float16)axis_q[(size_t)c * D + d];
    ENSURE(ctx->qt16, q16.size());
    HIPCHK(hipMemcpy(ctx->qt16.p, q16.data(), q16.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    ctx->Kq16 = Kq;
  }
  ctx->fmax_len = feature_max_len;
  if (feature_max_len > 0) {
    ENSURE(ctx->fmax, (size_t)feature_max_len);
    HIPCHK(hipMemcpy(ctx->fmax.p, feature_max, (size_t)feature_max_len * 4, hipMemcpyHostToDevice));
  }
  ctx->h_axis_p.assign(axis_p ? axis_p : nullptr, axis_p ? axis_p + (size_t)D * F : nullptr);
  ctx->h_var.assign(var ? var : nullptr, var ? var + D : nullptr);
  ctx->h_axis_q.assign(axis_q, axis_q + (size_t)M * r * D);
  ctx->h_fmax.assign(feature_max ? feature_max : nullptr,
                     feature_max ? feature_max + feature_max_len : nullptr);
  ++ctx->setup_version;
  ctx->compress = axis_p != nullptr;
  ctx->D = D;
  ctx->D_user = D_user;
  ctx->F = F;
  ctx->M = M;
  ctx->r = r;
  ctx->Dpad = Dpad;
  ctx->have_setup = true;
  ctx->g_valid = false;
  if (ctx->lists.M != M) init_lists(ctx);
  return C3H_OK;
}

int c3h_search_setup(c3h_ctx* ctx, const float* axis_p, const float* var, int32_t D, int32_t F,
                     const float* axis_q, int32_t M, int32_t r, const float* feature_max,
                     int32_t feature_max_len) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (D < 1 || F < 1 || M < 1 || r < 1 || !axis_q || feature_max_len < 0 ||
      (feature_max_len > 0 && !feature_max))
    return fail(ctx, C3H_ERR_ARG, "c3h_search_setup: bad arguments");
  if (!axis_p && D != F)
    return fail(ctx, C3H_ERR_ARG, "c3h_search_setup: without compression D must equal F");
  if (D % 4 == 0 || D > 160)
    return search_setup_dev(ctx, axis_p, var, D, F, axis_q, M, r, feature_max, feature_max_len, D);
  // the sparse search, the pipeline and the matrix-core projection take D in 4-float chunks:
  // zero axes (unit variance) are appended.  Their compressed values are 0, so every dot
  // product and norm adds exact zeros: the scores are the caller's D's, bit for bit
  const int Dp = (D + 3) / 4 * 4;
  std::vector<float> ap, vp((size_t)Dp, 1.0f), qp((size_t)M * r * Dp, 0.0f);
  if (axis_p) {  // (identity compression, D == F: the appended axes select no bin)
    ap.assign((size_t)Dp * F, 0.0f);
    std::copy(axis_p, axis_p + (size_t)D * F, ap.begin());
  }
  if (var) std::copy(var, var + D, vp.begin());
  for (int c = 0; c < M * r; ++c) std::copy(axis_q + (size_t)c * D, axis_q + (size_t)(c + 1) * D, qp.begin() + (size_t)c * Dp);
  return search_setup_dev(ctx, axis_p ? ap.data() : nullptr, var ? vp.data() : nullptr, Dp, F, qp.data(), M, r,
                          feature_max, feature_max_len, D);
}

int c3h_set_rank(c3h_ctx* ctx, int32_t rank) {
  if (!ctx || rank < 1 || rank > 4096) return C3H_ERR_ARG;
  QUIESCE(ctx);
  ctx->rank = rank;
  init_lists(ctx);
  return C3H_OK;
}

int c3h_clean_max(c3h_ctx* ctx) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (ctx->lists.M != std::max(ctx->M, 1) || ctx->lists.rank != ctx->rank) init_lists(ctx);
  if (ctx->lists_dev_valid) {
    // the device copy is current: the next replay kernel applies the clean (or the next
    // download), so the next search uploads nothing -- the per-callback loop's cleanData
    // then costs no H2D copy on the frame's critical path (round 6).  A host copy that is
    // current takes the clean too.
    ctx->pending_clean = true;
    if (ctx->lists_host_valid) {
      auto& L = ctx->lists;
      std::fill(L.score.begin(), L.score.end(), 0.0);
      std::fill(L.x.begin(), L.x.end(), 0);
      std::fill(L.y.begin(), L.y.end(), 0);
      std::fill(L.z.begin(), L.z.end(), 0);
    }
    return C3H_OK;
  }
  auto& L = ctx->lists;
  std::fill(L.score.begin(), L.score.end(), 0.0);
  std::fill(L.x.begin(), L.x.end(), 0);
  std::fill(L.y.begin(), L.y.end(), 0);
  std::fill(L.z.begin(), L.z.end(), 0);
  ctx->lists_dev_valid = false;
  return C3H_OK;
}

int c3h_search(c3h_ctx* ctx, const int32_t range[3], int32_t exist_threshold, int32_t rotate,
               int32_t remove_overlap, c3h_det* out) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  HIPCHK(hipSetDevice(ctx->device));
  const int nm = run_search(ctx, range, exist_threshold, rotate, nullptr);
  if (nm < 0) return nm;
  int rc = sync_host_lists(ctx);
  if (rc != C3H_OK) return rc;
  auto& L = ctx->lists;
  const size_t n = (size_t)L.M * L.rank;
  std::vector<c3h_det> recs(n);
  for (size_t i = 0; i < n; ++i) recs[i] = c3h_det{L.score[i], L.x[i], L.y[i], L.z[i], L.mode[i]};
  if (remove_overlap) {
    c3h_remove_overlap(L.M, L.rank, range, recs.data());
    for (size_t i = 0; i < n; ++i) {
      L.score[i] = recs[i].score;
      L.x[i] = recs[i].x;
      L.y[i] = recs[i].y;
      L.z[i] = recs[i].z;
      L.mode[i] = recs[i].mode;
    }
    ctx->lists_dev_valid = false;
  }
  if (out) memcpy(out, recs.data(), n * sizeof(c3h_det));
  return nm;
}

int c3h_search_async(c3h_ctx* ctx, const int32_t range[3], int32_t exist_threshold,
                     int32_t rotate, c3h_det* d_out) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  HIPCHK(hipSetDevice(ctx->device));
  const int nm = run_search(ctx, range, exist_threshold, rotate, d_out);
  if (nm < 0) return nm;
  if (nm == 0 && d_out) {  // no search ran: hand out the current lists
    int rc = sync_host_lists(ctx);
    if (rc != C3H_OK) return rc;
    rc = upload_lists(ctx);
    if (rc != C3H_OK) return rc;
    const size_t n = (size_t)ctx->lists.M * ctx->lists.rank;
    HIPCHK(hipMemcpyAsync(d_out, ctx->d_lists.p, n * sizeof(c3h_det), hipMemcpyDeviceToDevice, ctx->stream));
  }
  return nm;
}

int c3h_set_lanes(c3h_ctx* ctx, int32_t lanes) {
  if (!ctx || lanes < 1 || lanes > 16) return C3H_ERR_ARG;
  ctx->nlanes = lanes;
  return C3H_OK;
}

int c3h_set_batch(c3h_ctx* ctx, int32_t frames) {
  if (!ctx || frames < 1 || frames > c3h::kMaxBatch) return C3H_ERR_ARG;
  QUIESCE(ctx);
  ctx->nbatch = frames;
  return C3H_OK;
}

}  // extern "C"

namespace {

// child contexts lanes[0 .. n-1] exist and carry the context's search setup and rank
int ensure_lanes(c3h_ctx* ctx, int n) {
  while ((int)ctx->lanes.size() < n) {
    c3h_ctx* c = nullptr;
    int rc = c3h_create(ctx->device, &c);
    if (rc != C3H_OK) return fail(ctx, rc, "c3h_run_frames: lane context");
    c->parent = ctx;
    ctx->lanes.push_back(c);
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->lane_ev.push_back(e);
  }
  bool synced = false;
  for (int l = 0; l < n; ++l) {
    c3h_ctx* c = ctx->lanes[l];
    if (c->setup_version != ctx->setup_version || !c->have_setup) {
      if (!synced) {  // pipelined batches of this lane may still be queued on the parent's stream
        HIPCHK(hipStreamSynchronize(ctx->stream));
        synced = true;
      }
      int rc = search_setup_dev(c, ctx->h_axis_p.empty() ? nullptr : ctx->h_axis_p.data(),
                                ctx->h_var.empty() ? nullptr : ctx->h_var.data(), ctx->D, ctx->F,
                                ctx->h_axis_q.data(), ctx->M, ctx->r,
                                ctx->h_fmax.empty() ? nullptr : ctx->h_fmax.data(), (int)ctx->h_fmax.size(),
                                ctx->D_user);
      if (rc != C3H_OK) return fail(ctx, rc, std::string("c3h_run_frames: lane setup: ") + c->err);
      c->setup_version = ctx->setup_version;
    }
    if (c->rank != ctx->rank) {
      int rc = c3h_set_rank(c, ctx->rank);
      if (rc != C3H_OK) return rc;
    }
  }
  return C3H_OK;
}

// frames of chunk ch (B per chunk); the last chunk puts its last frame in slot 0, so the
// context that runs it ends up holding the last frame's state
int chunk_frames(const uint32_t* const* d_grids, c3h_det* d_out, size_t per_frame, int nframes, int B,
                 int nchunks, int ch, const uint32_t** grids, c3h_det** outs) {
  const int f0 = ch * B, nb = std::min(B, nframes - f0);
  for (int j = 0; j < nb; ++j) {  // nchunks < 0: natural order throughout
    const int fi = (ch == nchunks - 1) ? (j == 0 ? f0 + nb - 1 : f0 + j - 1) : f0 + j;
    grids[j] = d_grids[fi];
    outs[j] = d_out + (size_t)fi * per_frame;
  }
  return nb;
}

// Software-pipelined batches (pipeline.hip).  Batch number s is prepared on buffer set
// s % 4 (set 0 = this context) and runs as the occupancy role of one tick, the tile role
// of the next, compress+gate of the one after and scoring + rank-1 argmax of the fourth.
// All buffer sets work on this context's stream, so ticks order themselves; the host
// only enqueues.  The pipeline persists across c3h_stream_frames calls (a continuous
// frame source keeps it full); c3h_run_frames and c3h_stream_flush drain it.
constexpr int kPipeDepth = 4;

c3h_ctx* pipe_set(c3h_ctx* ctx, uint64_t seq) {
  const int set = (int)(seq % kPipeDepth);
  return set == 0 ? ctx : ctx->lanes[set - 1];
}

// lane contexts enqueue on the parent's stream while a pipeline call runs
struct PipeScope {
  c3h_ctx* ctx;
  hipStream_t saved[kPipeDepth - 1];
  explicit PipeScope(c3h_ctx* c) : ctx(c) {
    ctx->pipe_busy = true;
    for (int l = 0; l < kPipeDepth - 1 && l < (int)ctx->lanes.size(); ++l) {
      saved[l] = ctx->lanes[l]->stream;
      ctx->lanes[l]->stream = ctx->stream;
    }
  }
  ~PipeScope() {
    for (int l = 0; l < kPipeDepth - 1 && l < (int)ctx->lanes.size(); ++l) ctx->lanes[l]->stream = saved[l];
    ctx->pipe_busy = false;
  }
};

// one tick: the occupancy role of `fresh` (nullable) and the next role of every batch in
// flight; afterwards every batch is one stage older and finished batches leave
int pipe_tick(c3h_ctx* ctx, const c3h_ctx::PipeBatch* fresh) {
  c3h::TickParts tp;
  tp.prof = &ctx->prof;
  if (fresh && !fresh->stamped) tp.occ = &fresh->l;
  for (auto& b : ctx->pipe) {
    if (b.age == 1) tp.tile = &b.l;
    if (b.age == 2) {
      tp.gate = &b.q;
      tp.comp = &b.sc;
    }
    if (b.age == 3) tp.score = &b.q;
  }
  {
    Timed tm(ctx, 5, fresh ? fresh->nf : 0);
    hipError_t e = c3h::launch_tick(tp, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, "launch_tick", e);
  }
  for (auto& b : ctx->pipe) {
    if (b.age == 2 && b.set) b.set->scores_layout = b.layout;  // this tick enqueued its gate
    if (b.age == 1 && b.fix) {  // its tile role ran in this tick: the off-cell fixup before its compress
      hipError_t e = c3h::launch_point_fixup(b.fx, ctx->stream);
      if (e != hipSuccess) return hip_fail(ctx, "launch_point_fixup", e);
    }
  }
  std::vector<c3h_ctx::PipeBatch> next;
  for (auto& b : ctx->pipe)
    if (b.age < 3) {
      next.push_back(b);
      next.back().age++;
    }
  if (fresh) {
    next.push_back(*fresh);
    next.back().age = 1;
  }
  ctx->pipe.swap(next);
  return C3H_OK;
}

int pipe_flush(c3h_ctx* ctx) {
  if (ctx->pipe.empty()) return C3H_OK;
  PipeScope scope(ctx);
  while (!ctx->pipe.empty()) {
    int rc = pipe_tick(ctx, nullptr);
    if (rc != C3H_OK) {
      ctx->pipe.clear();
      return rc;
    }
  }
  return C3H_OK;
}

// public entry points that touch this context's buffers drain an open stream first
int pipe_quiesce(c3h_ctx* ctx) {
  if (ctx->pipe_busy || ctx->pipe.empty()) return C3H_OK;
  return pipe_flush(ctx);
}

// Captures nb frames as the next batch on its buffer set (no launch: its tile stamps may
// come from elsewhere first).  Returns > 0 (modes searched), 0 when the configuration does
// not fit the tick (only possible for the first batch of a stream: the caller then runs
// the lanes), < 0 on error.
int pipe_prepare(c3h_ctx* ctx, const uint32_t* const* grids, c3h_det* const* outs, int nb,
                 const c3h_ctx::PipeKey& k, const int32_t* lim, c3h_ctx::PipeBatch* fresh) {
  c3h_ctx* c = pipe_set(ctx, ctx->pipe_seq);
  c->capture = true;
  c->cap_c3_valid = c->cap_search_valid = false;
  int rc = c3h_set_grid(c, grids[0], k.div_b, k.min_b, k.leaf, 1);
  if (rc == C3H_OK) rc = extract_frames(c, grids, nb, &k.p, nullptr, nullptr);
  if (rc == C3H_OK) rc = search_frames(c, nb, k.range, k.thr, k.rotate, outs, 2);
  c->capture = false;
  c->cap_q.lim = lim;  // canvas frames: each frame's own subdivisions bound its positions
  if (rc < 0) {
    if (c != ctx) ctx->err = c->err;
    return rc;
  }
  const bool fits = c->cap_c3_valid && c->cap_search_valid && c->cap_sparse_g && c->cap_argmax &&
                    c3h::tick_ok(c->cap_c3);
  if (!fits) {  // one geometry per stream: decided on its first batch
    if (!ctx->pipe.empty()) return fail(ctx, C3H_ERR_STATE, "pipeline: internal: geometry changed");
    return 0;
  }
  c->nframes_feat = 1;  // slot 0 is the context's view from here on
  *fresh = c3h_ctx::PipeBatch{c->cap_c3, c->cap_q, c->cap_sc, nb, 0};
  fresh->set = c;
  fresh->layout = c->cap_layout;
  return rc;
}

// Launches a prepared batch's first tick; rc: pipe_prepare's result (> 0)
int pipe_commit(c3h_ctx* ctx, const c3h_ctx::PipeBatch& fresh, const c3h_ctx::PipeKey& k, int rc) {
  if (ctx->pipe.empty()) {
    // a stream starts: the occupancy role's tail-stealing pool (words 0-1 of each buffer
    // set's tile flags) resets itself at the end of every launch; zero it here as well, so
    // a launch that ended early (an aborted stream) cannot leave it counting
    for (int sidx = 0; sidx < kPipeDepth; ++sidx) {
      c3h_ctx* c = sidx == 0 ? ctx : (sidx - 1 < (int)ctx->lanes.size() ? ctx->lanes[sidx - 1] : nullptr);
      if (c && c->tileflags.p && c->tileflags.n >= 2)
        HIPCHK(hipMemsetAsync(c->tileflags.p, 0, 2 * sizeof(uint32_t), ctx->stream));
    }
  }
  int trc = pipe_tick(ctx, &fresh);
  if (trc != C3H_OK) return trc;
  ctx->pipe_seq++;
  ctx->pipe_key = k;
  ctx->pipe_nm = rc;
  return rc;
}

// Prepares nb frames as the next batch on its buffer set and launches its first tick.
// Returns as pipe_prepare.
int pipe_push(c3h_ctx* ctx, const uint32_t* const* grids, c3h_det* const* outs, int nb,
              const c3h_ctx::PipeKey& k, const int32_t* lim = nullptr) {
  c3h_ctx::PipeBatch fresh{};
  const int rc = pipe_prepare(ctx, grids, outs, nb, k, lim, &fresh);
  if (rc <= 0) return rc;
  return pipe_commit(ctx, fresh, k, rc);
}

c3h_ctx::PipeKey pipe_key(c3h_ctx* ctx, const int32_t div_b[3], const int32_t min_b[3], float leaf,
                          const c3h_extract_params* p, const int32_t range[3], int32_t thr, int32_t rotate,
                          int B) {
  c3h_ctx::PipeKey k;
  memset(&k, 0, sizeof(k));  // compared bytewise
  memcpy(k.div_b, div_b, sizeof(k.div_b));
  memcpy(k.min_b, min_b, sizeof(k.min_b));
  k.leaf = leaf;
  k.p = *p;
  memcpy(k.range, range, sizeof(k.range));
  k.thr = thr;
  k.rotate = rotate ? 1 : 0;
  k.batch = B;
  k.rank = ctx->rank;
  k.setup_version = ctx->setup_version;
  return k;
}

bool pipelinable(const c3h_ctx* ctx) {
  return ctx->pipeline && ctx->rank == 1 && c3h::score_fast_ok(ctx->D, ctx->r);
}

// Runs nframes through the pipeline in batches of B.  drain: run the fill/drain ticks so
// every result is complete on return (c3h_run_frames); the last batch is then placed on
// set 0 with its last frame in slot 0, so this context holds the last frame's state.
// Returns as pipe_push.
int run_frames_pipelined(c3h_ctx* ctx, const uint32_t* const* d_grids, int32_t nframes,
                         const int32_t div_b[3], const int32_t min_b[3], float leaf,
                         const c3h_extract_params* p, const int32_t range[3], int32_t exist_threshold,
                         int32_t rotate, c3h_det* d_out, int B, bool drain) {
  const size_t per_frame = (size_t)std::max(ctx->M, 1) * ctx->rank;
  const int nchunks = (nframes + B - 1) / B;
  int rc = ensure_lanes(ctx, kPipeDepth - 1);
  if (rc != C3H_OK) return rc;
  const c3h_ctx::PipeKey k = pipe_key(ctx, div_b, min_b, leaf, p, range, exist_threshold, rotate, B);
  if (!ctx->pipe.empty() && memcmp(&k, &ctx->pipe_key, sizeof(k)) != 0) {
    rc = pipe_flush(ctx);  // a different stream: drain the open one first
    if (rc != C3H_OK) return rc;
  }
  PipeScope scope(ctx);
  if (drain && ctx->pipe.empty())  // the last batch lands on set 0
    ctx->pipe_seq = (uint64_t)((kPipeDepth - (nchunks - 1) % kPipeDepth) % kPipeDepth);
  int nm = 0;
  for (int ch = 0; ch < nchunks; ++ch) {
    const uint32_t* grids[c3h::kMaxBatch];
    c3h_det* outs[c3h::kMaxBatch];
    const int nb = chunk_frames(d_grids, d_out, per_frame, nframes, B, drain ? nchunks : -1, ch, grids, outs);
    rc = pipe_push(ctx, grids, outs, nb, k);
    if (rc <= 0) {
      if (rc == 0 && ch == 0) return 0;
      ctx->pipe.clear();
      return rc == 0 ? fail(ctx, C3H_ERR_STATE, "pipeline: internal: batch does not fit") : rc;
    }
    nm = rc;
  }
  if (drain) {
    while (!ctx->pipe.empty()) {
      rc = pipe_tick(ctx, nullptr);
      if (rc != C3H_OK) {
        ctx->pipe.clear();
        return rc;
      }
    }
  }
  return nm;
}

}  // namespace

extern "C" {

int c3h_run_frames(c3h_ctx* ctx, const uint32_t* const* d_grids, int32_t nframes,
                   const int32_t div_b[3], const int32_t min_b[3], float leaf,
                   const c3h_extract_params* p, const int32_t range[3], int32_t exist_threshold,
                   int32_t rotate, c3h_det* d_out) {
  if (!ctx || !d_grids || nframes < 0 || !div_b || !min_b || !p || !range || !d_out)
    return C3H_ERR_ARG;
  if (!ctx->have_setup) return fail(ctx, C3H_ERR_STATE, "c3h_run_frames: no axes (call c3h_search_setup)");
  if (!extract_params_ok(p)) return fail(ctx, C3H_ERR_ARG, "c3h_run_frames: variant / color_mode");
  HIPCHK(hipSetDevice(ctx->device));
  {
    int rc = pipe_flush(ctx);  // an open stream completes first
    if (rc != C3H_OK) return rc;
  }
  if (nframes == 0) return 0;
  const size_t per_frame = (size_t)std::max(ctx->M, 1) * ctx->rank;
  // frames go in chunks of B (one set of launches per chunk, frame = launch y / z index)
  const int B = c3h::score_fast_ok(ctx->D, ctx->r) ? std::max(1, std::min(ctx->nbatch, c3h::kMaxBatch)) : 1;
  const int nchunks = (nframes + B - 1) / B;
  if (pipelinable(ctx)) {
    const int rc = run_frames_pipelined(ctx, d_grids, nframes, div_b, min_b, leaf, p, range, exist_threshold,
                                        rotate, d_out, B, true);
    if (rc != 0) return rc;
  }
  // lanes: chunks are spread over K child contexts on their own streams and host threads
  const int K = std::max(1, std::min(ctx->nlanes, nchunks));
  {
    int rc = ensure_lanes(ctx, K - 1);
    if (rc != C3H_OK) return rc;
  }
  if (!ctx->fork_ev) HIPCHK(hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ctx->fork_ev, ctx->stream));  // inputs were produced on ctx's stream
  for (int l = 0; l < K - 1; ++l) HIPCHK(hipStreamWaitEvent(ctx->lanes[l]->stream, ctx->fork_ev, 0));
  std::vector<int> lane_rc(K, 0);
  auto run_lane = [&](int lane) {
    c3h_ctx* c = lane == 0 ? ctx : ctx->lanes[lane - 1];
    if (lane) (void)hipSetDevice(c->device);
    int nm_lane = 0;
    for (int ch = 0; ch < nchunks; ++ch) {
      if ((nchunks - 1 - ch) % K != lane) continue;
      const uint32_t* grids[c3h::kMaxBatch];
      c3h_det* outs[c3h::kMaxBatch];
      const int nb = chunk_frames(d_grids, d_out, per_frame, nframes, B, nchunks, ch, grids, outs);
      int rc = c3h_set_grid(c, grids[0], div_b, min_b, leaf, 1);
      if (rc == C3H_OK) rc = extract_frames(c, grids, nb, p, nullptr, nullptr);
      if (rc == C3H_OK) rc = search_frames(c, nb, range, exist_threshold, rotate, outs, 2);
      if (rc < 0) {
        lane_rc[lane] = rc;
        return;
      }
      nm_lane = rc;
      c->nframes_feat = 1;  // slot 0 is the context's view from here on
    }
    lane_rc[lane] = nm_lane;
  };
  std::vector<std::thread> workers;
  for (int l = 1; l < K; ++l) workers.emplace_back(run_lane, l);
  run_lane(0);
  for (auto& w : workers) w.join();
  for (int l = 1; l < K; ++l)
    if (lane_rc[l] < 0) return fail(ctx, lane_rc[l], std::string("c3h_run_frames lane: ") + ctx->lanes[l - 1]->err);
  if (lane_rc[0] < 0) return lane_rc[0];
  for (int l = 0; l < K - 1; ++l) {  // join
    HIPCHK(hipEventRecord(ctx->lane_ev[l], ctx->lanes[l]->stream));
    HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->lane_ev[l], 0));
  }
  return lane_rc[0];
}

int c3h_stream_frames(c3h_ctx* ctx, const uint32_t* const* d_grids, int32_t nframes,
                      const int32_t div_b[3], const int32_t min_b[3], float leaf,
                      const c3h_extract_params* p, const int32_t range[3], int32_t exist_threshold,
                      int32_t rotate, c3h_det* d_out) {
  if (!ctx || !d_grids || nframes < 0 || !div_b || !min_b || !p || !range || !d_out)
    return C3H_ERR_ARG;
  if (!ctx->have_setup) return fail(ctx, C3H_ERR_STATE, "c3h_stream_frames: no axes (call c3h_search_setup)");
  if (!extract_params_ok(p)) return fail(ctx, C3H_ERR_ARG, "c3h_stream_frames: variant / color_mode");
  if (nframes == 0) return ctx->pipe_nm;
  HIPCHK(hipSetDevice(ctx->device));
  const int B = std::max(1, std::min(ctx->nbatch, c3h::kMaxBatch));
  if (pipelinable(ctx)) {
    const int rc = run_frames_pipelined(ctx, d_grids, nframes, div_b, min_b, leaf, p, range, exist_threshold,
                                        rotate, d_out, B, false);
    if (rc != 0) return rc;
  }
  // not pipelinable: the frames complete as in c3h_run_frames
  return c3h_run_frames(ctx, d_grids, nframes, div_b, min_b, leaf, p, range, exist_threshold, rotate, d_out);
}

int c3h_stream_flush(c3h_ctx* ctx) {
  if (!ctx) return C3H_ERR_ARG;
  HIPCHK(hipSetDevice(ctx->device));
  return pipe_flush(ctx);
}

}  // extern "C"

namespace {

// One frame on the single-frame path (c3h_voxelize + c3h_extract + search from the setRank
// state) into d_out_f: the frames c3h_run_point_frames' canvas cannot reproduce exactly.
int point_frame_single(c3h_ctx* ctx, const float* pts, int64_t n, int on_device, float leaf, float z_limit,
                       const c3h_extract_params* p, const int32_t range[3], int32_t thr, int32_t rotate,
                       c3h_det* d_out_f, c3h_frame_info* fi) {
  const size_t per_frame = (size_t)std::max(ctx->M, 1) * ctx->rank;
  HIPCHK(hipMemsetAsync(d_out_f, 0, per_frame * sizeof(c3h_det), ctx->stream));  // fresh lists
  c3h_grid_info gi{};
  int rc = c3h_voxelize(ctx, pts, n, on_device, leaf, z_limit, &gi);
  int32_t sb[3] = {0, 0, 0};
  if (rc == C3H_OK) rc = extract_frames(ctx, &ctx->grid_ptr, 1, p, sb, nullptr);
  if (rc == C3H_OK) rc = search_frames(ctx, 1, range, thr, rotate, &d_out_f, 2);
  if (fi) {
    memset(fi, 0, sizeof(*fi));
    if (rc >= 0) {
      for (int a = 0; a < 3; ++a) {
        fi->div_b[a] = gi.div_b[a];
        fi->min_b[a] = gi.min_b[a];
        fi->subdiv_b[a] = sb[a];
      }
      fi->n_valid = gi.n_valid;
      fi->n_occ = gi.n_occ;
    }
    fi->status = rc >= 0 ? 1 : rc;
  }
  return rc < 0 ? rc : C3H_OK;
}

}  // namespace

extern "C" {

// points-in batches: the scatter stamps the tick's tiles (0: the tick streams the canvases)
#ifndef C3H_POINT_STAMP
#define C3H_POINT_STAMP 1
#endif
constexpr bool kPointStamp = C3H_POINT_STAMP;
#ifndef C3H_POINT_VOX_PRIO
#define C3H_POINT_VOX_PRIO 1
#endif
// points-in batches: flagged voxels summed exactly and off-cell voxels fixed up in the batch
// (0: frames with flagged voxels take the single-frame path, as in round 3)
#ifndef C3H_POINT_EXACT
#define C3H_POINT_EXACT 1
#endif
constexpr bool kPointExact = C3H_POINT_EXACT;

int c3h_run_point_frames(c3h_ctx* ctx, const float* const* pts, const int64_t* n, int32_t nframes, int on_device,
                         float leaf, float z_limit, const int32_t canvas[3], const c3h_extract_params* p,
                         const int32_t range[3], int32_t exist_threshold, int32_t rotate, c3h_det* d_out,
                         c3h_frame_info* info) {
  if (!ctx || !pts || !n || nframes < 0 || !canvas || !p || !range || !d_out || !(leaf > 0)) return C3H_ERR_ARG;
  if (!ctx->have_setup) return fail(ctx, C3H_ERR_STATE, "c3h_run_point_frames: no axes (call c3h_search_setup)");
  for (int i = 0; i < nframes; ++i)
    if (n[i] < 0 || (n[i] > 0 && !pts[i]) || n[i] >= ((int64_t)1 << 24))
      return fail(ctx, C3H_ERR_ARG, "c3h_run_point_frames: frame point counts must be in [0, 16,777,215]");
  if (p->variant != 981 && p->variant != 117) return fail(ctx, C3H_ERR_ARG, "c3h_run_point_frames: variant");
  if (p->color_mode < C3H_COLOR_C3_FLOAT || p->color_mode > C3H_COLOR_CHLAC)
    return fail(ctx, C3H_ERR_ARG, "c3h_run_point_frames: color_mode");
  int64_t cvox = 1;
  for (int a = 0; a < 3; ++a) {
    if (canvas[a] < 1) return fail(ctx, C3H_ERR_ARG, "c3h_run_point_frames: canvas dims must be >= 1");
    cvox *= canvas[a];
  }
  if (cvox > 2147483647LL) return fail(ctx, C3H_ERR_RANGE, "c3h_run_point_frames: canvas beyond int32 voxel indices");
  HIPCHK(hipSetDevice(ctx->device));
  {
    int rc = pipe_flush(ctx);  // an open frame stream completes first
    if (rc != C3H_OK) return rc;
  }
  if (nframes == 0) return 0;
  const size_t per_frame = (size_t)std::max(ctx->M, 1) * ctx->rank;
  std::vector<c3h_frame_info> fi((size_t)nframes);
  std::vector<char> redo((size_t)nframes, 1);
  int nm = 0;
  std::vector<char> exact_ran((size_t)nframes, 0);  // per frame: its batch ran the exact pass + fixup
  // canvas subdivisions: a frame with one subdivision where the canvas has several takes the
  // single-frame path (computeC3HLAC's hist_num == 1 rule puts every voxel in histogram 0)
  bool canvas_multi = false;
  if (p->subdiv > 0) {
    const float inv_s = 1.0 / p->subdiv;
    int64_t hn = 1;
    for (int a = 0; a < 3; ++a) hn *= canvas[a] > p->offset[a] ? (int64_t)ceilf((canvas[a] - p->offset[a]) * inv_s) : 0;
    canvas_multi = hn > 1;
  }
  const bool batched = pipelinable(ctx) && p->subdiv >= 0 && p->thr[0] >= 0 && p->thr[1] >= 0 && p->thr[2] >= 0;
  if (batched) {
    const int B = std::max(1, std::min(ctx->nbatch, c3h::kMaxBatch));
    const int nchunks = (nframes + B - 1) / B;
    const int chunk = c3h::vb_chunk();
    int rc = ensure_lanes(ctx, kPipeDepth - 1);
    if (rc != C3H_OK) return rc;
    const int32_t zero[3] = {0, 0, 0};
    const c3h_ctx::PipeKey k = pipe_key(ctx, canvas, zero, leaf, p, range, exist_threshold, rotate, B);
    // shared: toroidal accumulators (one per frame slot; the scatter returns them to zero),
    // voxel lists, the frames' records, host staging
    // toroidal accumulator dims: powers of two >= the canvas (a frame whose extent fits the
    // canvas never wraps onto itself; the index is then three masks and shifts)
    int tb[3];
    int64_t tvox = 1;
    for (int a = 0; a < 3; ++a) {
      tb[a] = 0;
      while ((1 << tb[a]) < canvas[a]) ++tb[a];
      tvox <<= tb[a];
    }
    if (tvox > ((int64_t)1 << 31)) return fail(ctx, C3H_ERR_RANGE, "c3h_run_point_frames: canvas too large");
    if (ctx->pb_acc_vox != tvox || ctx->pb_acc_slots < B) {
      ENSURE(ctx->pb_acc, (size_t)B * tvox);
      ENSURE(ctx->pb_accM, (size_t)B * tvox);
      ENSURE(ctx->pb_fcnt, (size_t)c3h::kMaxBatch);
      HIPCHK(hipMemsetAsync(ctx->pb_acc.p, 0, (size_t)B * tvox * 16, ctx->stream));
      HIPCHK(hipMemsetAsync(ctx->pb_accM.p, 0xff, (size_t)B * tvox * 4, ctx->stream));
      HIPCHK(hipMemsetAsync(ctx->pb_fcnt.p, 0, (size_t)c3h::kMaxBatch * 4, ctx->stream));
      ctx->pb_acc_vox = tvox;
      ctx->pb_acc_slots = B;
    }
    ENSURE(ctx->pb_info, (size_t)nframes);
    // shared buffers sized for the largest batch up front: the voxeliser stream may still be
    // reading them while the next batch is prepared
    {
      int64_t max_blk = 1, max_pts = 1;
      for (int ch = 0; ch < nchunks; ++ch) {
        int64_t b = 0, q = 0;
        for (int j = ch * B; j < std::min(nframes, (ch + 1) * B); ++j) {
          b += std::max<int64_t>(1, (n[j] + chunk - 1) / chunk);
          q += n[j];
        }
        max_blk = std::max(max_blk, b);
        max_pts = std::max(max_pts, q);
      }
      if (max_blk > INT_MAX / chunk) return fail(ctx, C3H_ERR_RANGE, "c3h_run_point_frames: batch too large");
      ENSURE(ctx->pb_vlist, (size_t)max_blk * chunk);
      if (!on_device) ENSURE(ctx->pb_stage, (size_t)max_pts * 4);
    }
    if (!ctx->pb_vstream) {
      // the voxeliser's stream is the points-in call's critical path (its accumulate runs
      // beside the tick of the batches before, which has slack): high priority, so its
      // workgroups are dispatched first as CUs free up (C3H_POINT_VOX_PRIO 0: default)
      int lo = 0, hi = 0;
      if (C3H_POINT_VOX_PRIO && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && hi != lo)
        HIPCHK(hipStreamCreateWithPriority(&ctx->pb_vstream, hipStreamNonBlocking, hi));
      else
        HIPCHK(hipStreamCreateWithFlags(&ctx->pb_vstream, hipStreamNonBlocking));
    }
    if (!ctx->pb_vox_ev) HIPCHK(hipEventCreateWithFlags(&ctx->pb_vox_ev, hipEventDisableTiming));
    for (hipEvent_t& e : ctx->pb_tick_ev)
      if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // overlap pays where the tick is light: 512 x 128^3 frames 51k -> 74k frames/s.  While
    // the tick streamed the canvases, 256^3 lost with it (33k -> 30k: the 67 MB grid stream
    // and the voxeliser's atomics slowed each other down, profiles/r3/points_overlap/); with
    // the scatter's stamps (no canvas stream) it gains there too: 41k -> 45k frames/s
    // (profiles/r3/point_stamp/).  Canvases up to 2^25 voxels (256^3 and a little beyond)
#ifndef C3H_POINT_OVERLAP_VOX
#define C3H_POINT_OVERLAP_VOX (1 << 25)
#endif
    const bool overlap = cvox <= (int64_t)C3H_POINT_OVERLAP_VOX;
    const hipStream_t vs = overlap ? ctx->pb_vstream : ctx->stream;
    // every exit (errors included) leaves the voxeliser stream idle: the next call may
    // reallocate the buffers its work reads
    struct VsIdle {
      hipStream_t s;
      ~VsIdle() { (void)hipStreamSynchronize(s); }
    } vs_idle{vs};
    // the voxeliser stream starts after everything enqueued so far (the memsets above)
    HIPCHK(hipEventRecord(ctx->pb_vox_ev, ctx->stream));
    HIPCHK(hipStreamWaitEvent(vs, ctx->pb_vox_ev, 0));
    PipeScope scope(ctx);
    for (int ch = 0; ch < nchunks && rc >= 0; ++ch) {
      const int f0 = ch * B, nb = std::min(B, nframes - f0);
      c3h_ctx* c = pipe_set(ctx, ctx->pipe_seq);
      c3h::VoxBatchArgs va{};
      va.nf = nb;
      va.blk0[0] = 0;
      for (int j = 0; j < nb; ++j) {  // every frame at least one block: it publishes the record
        va.n[j] = n[f0 + j];
        va.blk0[j + 1] = va.blk0[j] + (int)std::max<int64_t>(1, (n[f0 + j] + chunk - 1) / chunk);
      }
      va.total = va.blk0[nb];
      // this set's buffers; a reallocation loses the previous batch's word lists, so the
      // canvas grids are then zeroed whole
      const int blk_cap = (int)std::min<int64_t>(c->pb_part.n / c3h::vox_part_words(), INT_MAX);
      if (c->pb_cvox != cvox || c->pb_slots < B || blk_cap < va.total) {
        // (re)allocation: nothing in flight may still use the set's old buffers
        HIPCHK(hipStreamSynchronize(vs));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        const int bc = std::max(va.total, blk_cap);
        ENSURE(c->pb_grid, (size_t)B * cvox);
        ENSURE(c->pb_lim, (size_t)B * 4);
        ENSURE(c->pb_part, (size_t)bc * c3h::vox_part_words());
        ENSURE(c->pb_wlist, (size_t)bc * chunk);
        ENSURE(c->pb_flags, (size_t)B * c3h::kVbFlagCap);
        ENSURE(c->pb_bucket, (size_t)B * c3h::kVbBucketCap);
        ENSURE(c->pb_moved, (size_t)B * c3h::kVbMovedCap);
        ENSURE(c->pb_xcnt, (size_t)B * 4);
        HIPCHK(hipMemsetAsync(c->pb_grid.p, 0, (size_t)B * cvox * 4, vs));
        c->pb_cvox = cvox;
        c->pb_slots = B;
        c->pb_prev_total = 0;
        c->pb_prev_nf = 0;
      }
      va.prev_nf = c->pb_prev_nf;
      va.prev_total = c->pb_prev_total;
      for (int j = 0; j <= c3h::kMaxBatch; ++j)
        va.prev_blk0[j] = j < (int)c->pb_prev_blk0.size() ? c->pb_prev_blk0[j] : va.prev_total;
      if (on_device) {
        for (int j = 0; j < nb; ++j) va.pts[j] = reinterpret_cast<const float4*>(pts[f0 + j]);
      } else {  // host frames: one staging copy per batch, ordered on the voxeliser stream
        int64_t o = 0;
        for (int j = 0; j < nb; ++j) {
          va.pts[j] = reinterpret_cast<const float4*>(ctx->pb_stage.p + 4 * o);
          if (n[f0 + j] > 0)
            HIPCHK(hipMemcpyAsync(ctx->pb_stage.p + 4 * o, pts[f0 + j], (size_t)n[f0 + j] * 16,
                                  hipMemcpyHostToDevice, vs));
          o += n[f0 + j];
        }
      }
      va.inv = 1.0f / leaf;
      va.leaf = leaf;
      va.z_limit = z_limit;
      for (int a = 0; a < 3; ++a) {
        va.C[a] = canvas[a];
        va.off[a] = p->subdiv > 0 ? p->offset[a] : 0;
      }
      va.subdiv = p->subdiv;
      va.inv_s = p->subdiv > 0 ? (float)(1.0 / p->subdiv) : 0.0f;
      for (int a = 0; a < 3; ++a) va.tb[a] = tb[a];
      va.acc = ctx->pb_acc.p;
      va.accM = ctx->pb_accM.p;
      va.s_acc = tvox;
      va.fcnt = ctx->pb_fcnt.p;
      va.vlist = ctx->pb_vlist.p;
      va.wlist = c->pb_wlist.p;
      va.part = c->pb_part.p;
      // every slot of the set: the previous batch on it may have had more frames than this one
      for (int j = 0; j < c3h::kMaxBatch; ++j)
        va.grid[j] = j < c->pb_slots ? c->pb_grid.p + (size_t)j * cvox : nullptr;
      if (va.prev_nf > c->pb_slots || va.nf > c->pb_slots)
        return fail(ctx, C3H_ERR_STATE, "c3h_run_point_frames: internal: frame slots");
      va.info = ctx->pb_info.p + f0;
      va.lim = c->pb_lim.p;
      const uint32_t* grids[c3h::kMaxBatch];
      c3h_det* outs[c3h::kMaxBatch];
      for (int j = 0; j < nb; ++j) {
        grids[j] = c->pb_grid.p + (size_t)j * cvox;
        outs[j] = d_out + (size_t)(f0 + j) * per_frame;
      }
      // the accumulate needs nothing of the batch's C3 launch, so it starts before the
      // launch is captured (the capture's host work, ~10 us, then runs beside it: a one-batch
      // call starts sooner).  The set's grids and gate limits were last read by the tick
      // pushed two batches ago (tile role: one tick after the batch's own, gate role: two),
      // so this batch's voxels overlap the previous batch's tick
      if (ch >= 2) HIPCHK(hipStreamWaitEvent(vs, ctx->pb_tick_ev[(ch - 2) & 3], 0));
      {
        Timed t(ctx, 0, nb, vs);
        HIPCHK(c3h::launch_vox_batch_accum(va, vs));
      }
      // until the chain below has run, the accumulators hold this batch's sums: an exit in
      // between has the next call re-zero them
      struct PbAccGuard {
        c3h_ctx* c;
        bool armed;
        ~PbAccGuard() {
          if (armed) c->pb_acc_vox = 0;
        }
      } pb_acc_guard{ctx, true};
      // the batch's launches are captured next: the scatter sets its tile stamps and work
      // lists (the occupancy stream's job), so its first tick carries no occupancy role and
      // no canvas is streamed (128^3: 8.4 MB, 256^3: 67 MB per frame)
      c3h_ctx::PipeBatch fresh{};
      const int h2d0 = c->cap_h2d;
      rc = pipe_prepare(ctx, grids, outs, nb, k, c->pb_lim.p, &fresh);
      if (rc == 0) rc = fail(ctx, C3H_ERR_STATE, "c3h_run_point_frames: the canvas does not fit the pipeline");
      if (rc < 0) break;
      const c3h::C3Launch& cl = fresh.l;
      va.stamp = (kPointStamp && cl.gx == canvas[0] && cl.gy == canvas[1] && cl.gz == canvas[2] &&
                  cl.ntiles <= ((int64_t)1 << 18)) ? 1 : 0;
      va.axmap = cl.axmap;
      va.ns0 = cl.nseg[0];
      va.ns1 = cl.nseg[1];
      va.ntiles = (int)cl.ntiles;
      va.epoch = cl.epoch;
      va.tf = cl.tf;
      va.work = cl.work;
      va.s_tf = cl.s_tf;
      va.s_work = cl.s_work;
      // the exact pass + off-cell fixup: the tick's direct mode (a row list, one tile per
      // subdivision) on the canvas itself; otherwise flagged frames take the single-frame path
      const bool exact = kPointExact && cl.rows && cl.axmap && cl.gx == canvas[0] && cl.gy == canvas[1] &&
                         cl.gz == canvas[2] && c3h::point_fixup_fits(cl.lmax);
      if (exact) {
        va.flags = c->pb_flags.p;
        va.bucket = c->pb_bucket.p;
        va.moved = c->pb_moved.p;
        va.xcnt = c->pb_xcnt.p;
        c3h::PointFixup& fx = fresh.fx;
        fx.nf = nb;
        for (int j = 0; j < nb; ++j) fx.grid[j] = grids[j];
        fx.moved = c->pb_moved.p;
        fx.xcnt = c->pb_xcnt.p;
        fx.info = ctx->pb_info.p + f0;
        for (int a = 0; a < 3; ++a) {
          fx.C[a] = canvas[a];
          fx.thr[a] = cl.thr[a];
        }
        fx.axmap = cl.axmap;
        fx.segs = cl.segs;
        fx.ns0 = cl.nseg[0];
        fx.ns1 = cl.nseg[1];
        fx.seg_stride = cl.seg_stride;
        fx.sbx = cl.sbx;
        fx.sby = cl.sby;
        fx.variant = cl.variant;
        fx.lut = cl.lut;
        fx.feat = cl.feat;
        fx.exist = cl.exist;
        fx.rows = cl.rows;
        fx.tf = cl.tf;
        fx.s_feat = cl.s_feat;
        fx.s_h = cl.s_h;
        fx.s_tf = cl.s_tf;
        fx.epoch = cl.epoch;
        for (int a = 0; a < 3; ++a) fx.lmax[a] = cl.lmax[a];
        fresh.fix = true;
      }
      if (exact) std::fill(exact_ran.begin() + f0, exact_ran.begin() + f0 + nb, (char)1);
      // tables / stamp resets the capture enqueued precede the stamps (first batches only)
      if (va.stamp && vs != ctx->stream && c->cap_h2d != h2d0) {
        HIPCHK(hipEventRecord(ctx->pb_vox_ev, ctx->stream));
        HIPCHK(hipStreamWaitEvent(vs, ctx->pb_vox_ev, 0));
      }
      {
        Timed t(ctx, 0, 0, vs);  // (the frames are counted with the accumulate)
        HIPCHK(c3h::launch_vox_batch_post(va, vs));
      }
      pb_acc_guard.armed = false;  // the scatter returns every touched accumulator to zero
      HIPCHK(hipEventRecord(ctx->pb_vox_ev, vs));
      c->pb_prev_nf = nb;
      c->pb_prev_total = va.total;
      c->pb_prev_blk0.assign(va.blk0, va.blk0 + nb + 1);
      fresh.stamped = va.stamp != 0;
      // A stamped batch has no role in its own first tick (that tick runs the tile role of
      // the batch before it, compress + gate and scoring of older ones), so the tick goes
      // ahead of this batch's voxeliser and only the next tick waits for it (round 6: the
      // batch's tile role then runs beside the next voxeliser instead of after it, one
      // tick less per call after the last voxeliser).  An unstamped batch's first tick
      // streams its canvases: it waits.
      if (!fresh.stamped) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->pb_vox_ev, 0));
      rc = pipe_commit(ctx, fresh, k, rc);
      if (rc > 0) nm = rc;
      if (rc >= 0) HIPCHK(hipEventRecord(ctx->pb_tick_ev[ch & 3], ctx->stream));
      if (fresh.stamped) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->pb_vox_ev, 0));
    }
    while (rc >= 0 && !ctx->pipe.empty()) {
      const int trc = pipe_tick(ctx, nullptr);
      if (trc != C3H_OK) rc = trc;
    }
    if (rc < 0) {
      ctx->pipe.clear();
      return rc;
    }
    // the records come back through pinned memory: one asynchronous copy and one stream
    // synchronisation (a pageable copy blocks, then the stream is synchronised again; ~20 us
    // of a 64-frame call's ~0.75 ms)
    if (ctx->h_recs_n < (size_t)nframes) {
      if (ctx->h_recs) HIPCHK(hipHostFree(ctx->h_recs));
      ctx->h_recs = nullptr;
      ctx->h_recs_n = 0;
      void* hp = nullptr;
      HIPCHK(hipHostMalloc(&hp, (size_t)nframes * sizeof(c3h::VoxFrameRec)));
      ctx->h_recs = static_cast<c3h::VoxFrameRec*>(hp);
      ctx->h_recs_n = (size_t)nframes;
    }
    const c3h::VoxFrameRec* recs = ctx->h_recs;
    HIPCHK(hipMemcpyAsync(ctx->h_recs, ctx->pb_info.p, (size_t)nframes * sizeof(c3h::VoxFrameRec),
                          hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < nframes; ++i) {
      const c3h::VoxFrameRec& r = recs[i];
      c3h_frame_info& o = fi[i];
      bool one = true;
      for (int a = 0; a < 3; ++a) {
        o.min_b[a] = r.min_b[a];
        o.div_b[a] = r.max_b[a] - r.min_b[a] + 1;
        o.subdiv_b[a] = r.sb[a];
        one = one && r.sb[a] == 1;
      }
      o.n_valid = r.n_valid;
      o.n_occ = r.n_occ;
      o.n_moved = (int32_t)r.moved;
      o.status = 0;
      const bool hist1_mismatch = p->subdiv > 0 && canvas_multi && one;
      const bool empty_sub = p->subdiv > 0 && (r.sb[0] == 0 || r.sb[1] == 0 || r.sb[2] == 0);
      redo[i] = (r.err || (r.flagged && !exact_ran[i]) || r.n_valid == 0 || hist1_mismatch || empty_sub) ? 1 : 0;
    }
  }
  for (int i = 0; i < nframes; ++i) {
    if (!redo[i]) continue;
    int rc = point_frame_single(ctx, pts[i], n[i], on_device, leaf, z_limit, p, range, exist_threshold, rotate,
                                d_out + (size_t)i * per_frame, &fi[i]);
    if (rc == C3H_ERR_HIP || rc == C3H_ERR_NOMEM) return rc;  // device trouble ends the call
  }
  if (!batched) {  // the modes the search schedules (search.cpp:384-417)
    int modes[6];
    nm = mode_schedule(range[0], range[1], range[2], rotate, modes);
  }
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (info) memcpy(info, fi.data(), fi.size() * sizeof(c3h_frame_info));
  return nm;
}

int c3h_set_pipeline(c3h_ctx* ctx, int32_t enable) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  ctx->pipeline = enable != 0;
  return C3H_OK;
}

int c3h_get_compressed(c3h_ctx* ctx, float* out, int on_device) {
  if (!ctx || !out) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (!ctx->g_valid) return fail(ctx, C3H_ERR_STATE, "no compressed features (run a search)");
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->D_user != ctx->D) {  // appended zero axes: the caller's D columns of each row
    const int W = ctx->D, Wu = ctx->D_user;
    const float* src = ctx->G.p;
    c3h::DevBuf<float> tmp;
    hipError_t e = hipSuccess;
    if (ctx->g_sparse) {  // rows of empty subdivisions were not written: 0
      int rc = ensure(ctx, tmp, (size_t)ctx->hist_num * W);
      if (rc != C3H_OK) return rc;
      e = c3h::launch_masked_rows(ctx->G.p, ctx->exist.p, ctx->hist_num, W, tmp.p, ctx->stream);
      src = tmp.p;
    }
    if (e == hipSuccess && ctx->hist_num > 0)
      e = hipMemcpy2DAsync(out, (size_t)Wu * 4, src, (size_t)W * 4, (size_t)Wu * 4, (size_t)ctx->hist_num,
                           on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    release(tmp);
    if (e != hipSuccess) return fail(ctx, C3H_ERR_HIP, std::string("c3h_get_compressed: ") + hipGetErrorString(e));
    return C3H_OK;
  }
  const size_t n = (size_t)ctx->hist_num * ctx->D;
  if (!ctx->g_sparse) {
    HIPCHK(hipMemcpyAsync(out, ctx->G.p, n * 4, on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return C3H_OK;
  }
  // sparse compress: rows of empty subdivisions (exist == 0) were not written; they are 0
  return masked_readback(ctx, ctx->G.p, ctx->D, out, on_device);
}

int c3h_get_scores(c3h_ctx* ctx, double* out, int64_t* n_out, int on_device) {
  if (!ctx) return C3H_ERR_ARG;
  QUIESCE(ctx);
  if (n_out) *n_out = ctx->scores_n;
  if (!out) return C3H_OK;
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->scores_n)
    HIPCHK(hipMemcpyAsync(out, ctx->scores.p, (size_t)ctx->scores_n * 8,
                          on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return C3H_OK;
}

int c3h_remove_overlap(int32_t M, int32_t rank, const int32_t range[3], c3h_det* lists) {
  if (M < 1 || rank < 1 || !range || !lists) return C3H_ERR_ARG;
  const int r1 = range[0], r2 = range[1], r3 = range[2];
  for (int m = 0; m < M; m++) {
    for (int i = 0; i < 1; i++) {
      for (int m2 = 0; m2 < M; m2++) {
        if (m2 == m) continue;
        c3h_det* Lm = lists + (size_t)m * rank;
        c3h_det* Lm2 = lists + (size_t)m2 * rank;
        const int ov = check_overlap(Lm2, rank, r1, r2, r3, Lm[i].x, Lm[i].y, Lm[i].z, Lm[i].mode);
        if (Lm[i].score > Lm2[ov].score)
          for (int j = ov; j < rank - 1; j++) Lm2[j] = Lm2[j + 1];
        else
          for (int j = i; j < rank - 1; j++) Lm[j] = Lm[j + 1];
      }
    }
  }
  return C3H_OK;
}

// searchPart's rank update (search.cpp:464-474 with checkOverlap :327-356) replayed on the
// host over c3h_get_scores-layout arrays: per scheduled mode, per model, positions in
// (z, y, x) scan order; a candidate reaches the update only above the current rank-th
// score (that score never decreases: the replay kernel's rule)
int c3h_replay_scores(int32_t M, int32_t rank, const int32_t range[3], int32_t rotate, const int32_t subdiv_b[3],
                      const double* scores, c3h_det* lists) {
  return c3h_replay_scores_floor(M, rank, range, rotate, subdiv_b, scores, lists, nullptr);
}

// the same, recording each row's entry floor: before the first position of row (mode, m,
// z, y), the model's rank-th score (row_floor layout: per searched mode, M x ze x ye)
int c3h_replay_scores_floor(int32_t M, int32_t rank, const int32_t range[3], int32_t rotate,
                            const int32_t subdiv_b[3], const double* scores, c3h_det* lists, double* row_floor) {
  if (M < 1 || rank < 1 || !range || !subdiv_b || !scores || !lists) return C3H_ERR_ARG;
  const int r1 = range[0], r2 = range[1], r3 = range[2];
  if (r1 < 1 || r2 < 1 || r3 < 1) return C3H_ERR_ARG;
  int modes[6];
  const int nm = mode_schedule(r1, r2, r3, rotate, modes);
  int64_t off = 0, roff = 0;
  int searched = 0;
  for (int i = 0; i < nm; ++i) {
    int xr, yr, zr;
    get_range(modes[i], r1, r2, r3, &xr, &yr, &zr);
    const int xe = subdiv_b[0] - xr + 1, ye = subdiv_b[1] - yr + 1, ze = subdiv_b[2] - zr + 1;
    if (!(xe > 0 && ye > 0 && ze > 0)) continue;
    const int64_t P = (int64_t)xe * ye * ze;
    for (int m = 0; m < M; ++m) {
      c3h_det* L = lists + (size_t)m * rank;
      const double* sc = scores + off + (int64_t)m * P;
      double* fl = row_floor ? row_floor + roff + (int64_t)m * ze * ye : nullptr;
      for (int64_t p = 0; p < P; ++p) {
        if (fl && p % xe == 0) fl[p / xe] = L[rank - 1].score;
        const double cs = sc[p];
        if (!(cs > L[rank - 1].score)) continue;
        const int x = (int)(p % xe), y = (int)((p / xe) % ye), z = (int)(p / ((int64_t)xe * ye));
        for (int j = 0; j < rank; j++) {
          if (cs > L[j].score) {
            const int num = check_overlap(L, rank, r1, r2, r3, x, y, z, modes[i]);
            for (int q = 0; q < num - j; q++) L[num - q] = L[num - 1 - q];
            if (j <= num) L[j] = c3h_det{cs, x, y, z, modes[i]};
            break;
          }
        }
      }
    }
    off += P * M;
    roff += (int64_t)M * ze * ye;
    ++searched;
  }
  return searched;
}

int c3h_pca_read(const char* path, int32_t ascii, float* axis, float* var, float* mean,
                 int32_t* has_mean, int32_t max_dim) {
  const bool query = !axis && !var;  // size query: read the header only
  if (!path || (!query && (!axis || !var))) return C3H_ERR_ARG;
  FILE* fp = fopen(path, ascii ? "r" : "rb");
  if (!fp) return C3H_ERR_NOTFOUND;
  int dim = -1;
  const bool got_dim = ascii ? fscanf(fp, "%d\n", &dim) == 1 : fread(&dim, sizeof(int), 1, fp) == 1;
  if (query) {
    fclose(fp);
    return got_dim && dim > 0 ? dim : C3H_ERR_FORMAT;
  }
  if (!got_dim || dim <= 0 || dim > max_dim) {
    fclose(fp);
    return C3H_ERR_FORMAT;
  }
  bool ok = true;
  for (int i = 0; i < dim && ok; i++)
    for (int j = 0; j < dim && ok; j++) {
      float* dst = &axis[(size_t)i * dim + j];  // axis(j, i): eigenvector i contiguous
      ok = ascii ? fscanf(fp, "%f ", dst) == 1 : fread(dst, sizeof(float), 1, fp) == 1;
    }
  for (int i = 0; i < dim && ok; i++)
    ok = ascii ? fscanf(fp, "%f\n", &var[i]) == 1 : fread(&var[i], sizeof(float), 1, fp) == 1;
  if (!ok) {
    fclose(fp);
    return C3H_ERR_FORMAT;
  }
  float t;
  const bool got = ascii ? fscanf(fp, "%f\n", &t) == 1 : fread(&t, sizeof(float), 1, fp) == 1;
  if (has_mean) *has_mean = got ? 1 : 0;
  if (got && mean) {
    mean[0] = t;
    for (int i = 1; i < dim; i++) {
      float v = 0;
      if (ascii ? fscanf(fp, "%f\n", &v) != 1 : fread(&v, sizeof(float), 1, fp) != 1) break;
      mean[i] = v;
    }
  }
  fclose(fp);
  return dim;
}

int c3h_timing(c3h_ctx* ctx, int32_t enable) {
  if (!ctx) return C3H_ERR_ARG;
  ctx->timer.mask = enable == 1 ? C3H_TIMING_ALL : (uint32_t)enable & C3H_TIMING_ALL;
  if (enable) {  // pre-create event pairs so no hipEventCreate lands in a timed region
    HIPCHK(hipSetDevice(ctx->device));
    while (ctx->timer.pool.size() < 2048) {
      hipEvent_t a, b;
      HIPCHK(hipEventCreate(&a));
      HIPCHK(hipEventCreate(&b));
      ctx->timer.pool.push_back({a, b});
    }
  }
  return C3H_OK;
}

int c3h_kernel_times(c3h_ctx* ctx, float* ms_out, int32_t* counts_out, int32_t reset) {
  if (!ctx) return C3H_ERR_ARG;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  std::lock_guard<std::mutex> g(ctx->timer.mu);
  for (int s = 0; s < C3H_NTIMERS; ++s) {
    for (auto& e : ctx->timer.pending[s]) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
        ctx->timer.ms[s] += ms;
        ctx->timer.count[s] += e.weight;
      }
      ctx->timer.pool.push_back({e.a, e.b});
    }
    ctx->timer.pending[s].clear();
  }
  for (int s = 0; s < C3H_NTIMERS; ++s) {
    if (ms_out) ms_out[s] = ctx->timer.ms[s];
    if (counts_out) counts_out[s] = ctx->timer.count[s];
    if (reset) {
      ctx->timer.ms[s] = 0;
      ctx->timer.count[s] = 0;
    }
  }
  return C3H_OK;
}

}  // extern "C"

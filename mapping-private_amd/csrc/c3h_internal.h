// c3h_internal.h -- context state and kernel-launcher declarations shared by the
// HIP translation units of libc3hlac_mi355x.so.  gfx950 only; no dual code paths.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/c3hlac_mi355x.h"

namespace c3h {

// packed colour/occupancy voxel word: 0 = empty, else kOcc | r<<16 | g<<8 | b
constexpr uint32_t kOcc = 1u << 24;
constexpr uint32_t kEmptyKey = 0xffffffffu;
constexpr int kBlock = 256;
// largest centre-voxel extent of one C3 tile per axis; subdivisions wider than this
// are split into several tiles whose exact integer partial sums are added in 64 bit.
constexpr int kTileMax = 16;

// reference constants (c3_hlac/src/c3_hlac.cpp:38-45), as float
constexpr float kNorm0 = 1 / 255.0;
constexpr float kNorm1 = 1 / 65025.0;
constexpr float kNorm117_1 = 1 / 845325.0;
constexpr float kNorm117_1Bin = 1 / 13.0;

// ---- device buffers --------------------------------------------------------------
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;  // capacity in elements
};

struct SearchLists {  // SearchObjMulti max_*_multi state, host side
  int rank = 0, M = 0;
  std::vector<double> score;
  std::vector<int32_t> x, y, z, mode;
};

struct ScorePartial {
  double score;
  int64_t order;  // (mode index << 40) | position, -1 = none
};

struct TimedPair {
  hipEvent_t a, b;
  int weight;  // frames the bracketed launches processed
};

struct Timer {
  std::mutex mu;  // lanes enqueue from their own host threads
  std::vector<TimedPair> pending[C3H_NTIMERS];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  float ms[C3H_NTIMERS] = {};
  int count[C3H_NTIMERS] = {};
  uint32_t mask = 0;  // slots being timed
};

}  // namespace c3h

namespace c3h {

// Workgroup barrier for LDS-only hand-offs: waits for this wave's LDS (and scalar) ops
// but not for its outstanding global loads/stores, so prefetches issued before the
// barrier stay in flight (__syncthreads() also drains vmcnt on gfx9).
__device__ __forceinline__ void lds_barrier() {
  __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Diagnostics knobs read from the environment (dispatch order, role sizes, per-block
// timestamps) exist only in diagnostics builds (make DIAG=1 -> -DC3H_DIAG); the product
// library ignores the environment.
inline const char* diag_env(const char* name) {
#ifdef C3H_DIAG
  const char* v = getenv(name);
  return v && *v ? v : nullptr;
#else
  (void)name;
  return nullptr;
#endif
}

// ---- launchers (defined in the .hip files) ----------------------------------------
// voxeliser (voxelize.hip): counters are uint32 words of VoxArgs::cnt
enum {
  kVcMin = 0,     // int32[3] min cell
  kVcMax = 3,     // int32[3] max cell
  kVcValid = 6,   // u64 valid points
  kVcSlots = 8,   // [2] occupied voxels (owning entries) of the frame of each epoch parity
  kVcFlag = 10,   // voxels whose centroid may leave their cell
  kVcErr = 11,    // kVcErrRange | kVcErrWrap
  kVcOver = 12,   // grid buffer too small (scatter not run)
  kVcOff = 13,    // off-cell voxels recorded by the exact pass
  kVcWords = 16
};
constexpr uint32_t kVcErrRange = 1;  // cell coordinates beyond +-2^20
constexpr uint32_t kVcErrWrap = 4;   // the frame's extent exceeds the toroidal accumulator (the
                                     // frame runs again on larger dims; the scatter wrote nothing)
// a listed voxel outside the frame's bounds, a point whose voxel has no owning entry of this
// frame, or a voxel whose accumulated count differs from the points filed into its bucket:
// the accumulators held sums the frame did not add.  Every such access is skipped (device-
// side bound checks) and the call fails (round 6: the round-5 fault)
constexpr uint32_t kVcErrBad = 8;
// toroidal accumulator cells at most 2^kVoxTorMaxBits (24 B each: 1.6 GB); a frame whose
// extent needs more is voxelised by sorting its points (launch_vox_sorted)
constexpr int kVoxTorMaxBits = 26;
// Single-frame voxeliser state.  The accumulators are toroidal: voxel (x, y, z) sums at
// t = (x mod 2^tb0) | (y mod 2^tb1) << tb0 | (z mod 2^tb2) << (tb0 + tb1), so a frame whose
// extent fits 2^tb per axis maps its voxels one-to-one without a hash table.  Every
// (accumulate block, voxel) pair adds its sums (the first toucher, seen by its returning
// add, lists the voxel); the scatter converts each listed voxel and returns its
// accumulator to zero.
struct VoxArgs {
  const float4* pts;
  int64_t n;
  float z_limit, inv, leaf;
  ulonglong2* acc;          // [2^(tb0+tb1+tb2)] {count << 40 | sum r, sum b << 32 | sum g}, 0 between frames
  uint32_t* mg;             // [same] min near-face margin (float bits) of the voxel's points, ~0 between frames
  uint32_t* tpos;           // [same] list position of the voxel's owning entry (written by the scatter)
  int tb[3];
  uint32_t* lists;          // [entries parity 0 | entries parity 1 | grid words parity 0 | parity 1] x lcap,
  uint64_t lcap;            //   each a segment of vox_positions(1) per accum block
  uint32_t* lcnt;           // [lcap] this frame's owning entries' point counts (0: not owning)
  int32_t* part;            // per parity, per accum block: bounds, counts (vox_part_words() ints)
  int nblk, nblk_prev, nblk_cap;  // accum blocks of this / the previous frame, capacity
  uint32_t* cnt;            // kVcWords counters (totals published by the scatter)
  uint32_t* grid;           // packed grid buffer (capacity grid_cap words)
  int64_t grid_cap;
  int par;                  // epoch parity of this frame
  int clear_grid;           // clear the grid words the previous frame listed
  int blk0;                 // first accumulate block of this launch (chunked host input)
  long long* prof;          // diagnostics builds only (C3H_PROF): per-block phase timestamps
};
hipError_t launch_voxelize(const VoxArgs& a, hipStream_t s);
// the accumulate pass over blocks [a.blk0, a.blk0 + nblocks) only (host frames copied in
// chunks: each chunk's blocks start when its copy lands; the first launch (blk0 0) resets
// the counters and clears the previous frame's words)
hipError_t launch_vox_accum(const VoxArgs& a, int nblocks, hipStream_t s);
// f16 feature rows -> f32 rows when *flag (device-side check: no host sync)
hipError_t launch_feat16_to_f32(const _Float16* f16, int f16s, const uint32_t* flag, int64_t H, int F, float* out,
                                hipStream_t s);
hipError_t launch_vox_scatter(const VoxArgs& a, hipStream_t s);
int64_t vox_blocks(int64_t n);
int64_t vox_positions(int64_t n);
int vox_part_words();
constexpr int kVoxPartNew = 7;  // a partial record's word holding its segment's entry count
hipError_t launch_vox_centroids(const VoxArgs& a, uint32_t* counts, uint32_t* offs, uint32_t* cur,
                                uint32_t* block_sums, uint32_t* bucket, float4* cent, int32_t* offcell,
                                hipStream_t s);
hipError_t launch_vox_downsampled(const VoxArgs& a, const float4* cent, const uint32_t* counts, const int32_t* leaf,
                                  float* out, hipStream_t s);
hipError_t launch_vox_clear(const VoxArgs& a, hipStream_t s);
// wide frames (extent beyond 2^kVoxTorMaxBits accumulator cells): the voxeliser by a stable
// radix sort of (voxel index, point index) pairs.  mn / dv: the frame's bounds from the first
// pass; nv: its valid points.  Writes the grid, the lists, counts, exact centroids and the
// off-cell records (the state the exact pass would leave).  tmp_bytes query: tmp == nullptr.
struct VoxSortBufs {
  uint32_t *keys, *keys2, *idx, *idx2, *head, *block_sums;
  int32_t* ord;
  void* tmp;
  size_t tmp_bytes;
};
hipError_t launch_vox_sorted(const VoxArgs& a, const int mn[3], const int dv[3], int64_t nv, VoxSortBufs& b,
                             uint32_t* counts, float4* cent, int32_t* offcell, hipStream_t s);
int64_t scan_blocks(int64_t n);
hipError_t launch_leaf_layout(const uint32_t* grid, int64_t nvox, int32_t* leaf,
                              uint32_t* block_sums, int64_t nblocks, hipStream_t s);

#ifndef C3H_MAX_BATCH
#define C3H_MAX_BATCH 64
#endif
constexpr int kMaxBatch = C3H_MAX_BATCH;  // frames per launch (blockIdx.y) in c3h_run_frames

// ---- batched voxeliser (c3h_run_point_frames, voxelize.hip) --------------------------
// Frames of one batch are voxelised together, each into a fixed "canvas" grid of C^3 words
// placed at the frame's own min_b (canvas index = cell - min_b, so subdivisions, neighbours
// and box positions are the frame's own).  Per frame a toroidal accumulator of C^3 entries
// (cell coordinates mod C) replaces the hash table: cells of a frame whose extent fits the
// canvas never collide.  Per-frame results the host reads back once per call:
struct VoxFrameRec {
  int32_t min_b[3], max_b[3];
  int32_t sb[3];        // the frame's own getSubdivNum (the gate's position limits)
  uint32_t n_valid, n_occ;
  uint32_t flagged;     // voxels whose centroid may round across their cell boundary
  uint32_t err;         // bit 0: cell coordinates beyond +-2^20; bit 1: extent beyond the canvas;
                        // bit 2: flagged voxels beyond the exact pass's capacity; bit 3: a
                        // centroid cell past the last subdivision (the reference reads out of bounds)
  uint32_t moved;       // voxels whose exact centroid lies in another cell (the fixup's)
};
// exact-centroid pass of the batched voxeliser (round 4): per frame, the voxels the scatter
// flagged (their points are bucketed and summed in input order), and those whose centroid
// cell differs from their own cell
constexpr int kVbFlagCap = 4096;        // flagged voxels per frame
constexpr int kVbBucketCap = 1 << 16;   // their points per frame
constexpr int kVbMovedCap = 256;        // off-cell voxels per frame
struct VoxFlag {
  uint32_t t;       // toroidal accumulator key
  uint32_t idx;     // canvas word index
  uint32_t count;   // points
  uint32_t off;     // first bucket word
  uint32_t cur;     // bucket fill (atomic)
  uint32_t pad;
};
struct VoxMoved {
  uint32_t idx;     // canvas word index of the voxel's own cell
  int32_t base[3];  // canvas coordinates of its centroid's cell (floor(c / leaf) - min_b)
};
static_assert(sizeof(VoxMoved) == 16, "VoxMoved: 4 words (point_fixup_kernel's LDS layout)");
struct VoxBatchArgs {
  int nf, total;                      // frames, accumulate blocks of this batch
  int prev_nf, prev_total;            // the previous batch on this buffer set (its words to clear)
  const float4* pts[kMaxBatch];
  int64_t n[kMaxBatch];
  int blk0[kMaxBatch + 1];            // accumulate blocks of frame f: [blk0[f], blk0[f+1])
  int prev_blk0[kMaxBatch + 1];
  float inv, leaf, z_limit;
  int C[3];                           // canvas dims
  int tb[3];                          // toroidal accumulator: 2^tb[a] >= C[a] cells per axis
  int subdiv, off[3];
  float inv_s;
  ulonglong2* acc;                    // [frame][2^(tb0+tb1+tb2)] {count << 40 | sum r, sum b << 32 | sum g}
  uint32_t* accM;                     //                min boundary margin (float bits), ~0 = none
  int64_t s_acc;
  uint32_t* fcnt;                     // [kMaxBatch] finished accumulate blocks per frame (self-resetting)
  uint32_t* vlist;                    // [block][chunk] the block's (block, voxel) entries (toroidal index)
  uint32_t* wlist;                    // [block][chunk] canvas words the scatter wrote (this set)
  int32_t* part;                      // [block][kPartW] partial records (this set)
  uint32_t* grid[kMaxBatch];          // canvas grids of this set's frame slots (all slots)
  VoxFrameRec* info;                  // [nf]
  int32_t* lim;                       // [nf][4]: the frame's subdivisions per axis (0 = none)
  // tile stamps of the tick's occupancy role, set by the scatter instead (stamp = 1): the
  // tick then skips the occupancy stream over these canvases (OccArgs of the batch's C3 launch)
  int stamp;
  const int16_t* axmap;               // [C0 + C1 + C2] voxel coordinate -> subdivision (-1: none)
  int ns0, ns1;                       // subdivisions along x, y
  int ntiles;                         // subdivisions of the canvas (<= 2^18: an LDS bitmap)
  uint32_t epoch;
  uint32_t* tf;                       // per frame: [2] reserved | [2] work counters | stamps
  int32_t* work;                      // per frame: the non-empty tile list
  int64_t s_tf, s_work;
  // exact pass (nullable: flagged frames then take the single-frame path)
  VoxFlag* flags;                     // [nf][kVbFlagCap]
  uint32_t* bucket;                   // [nf][kVbBucketCap] point indices
  VoxMoved* moved;                    // [nf][kVbMovedCap]
  uint32_t* xcnt;                     // [nf][4]: flags, bucket words, moved, - (zeroed by voxb_reduce)
};
int vb_chunk();  // points per accumulate block
// The off-cell correction of a points-in batch, run after the tick that ran the batch's
// tile role and before the one that compresses it: every subdivision holding a voxel the
// exact pass moved (its own cell's and its centroid cell's) is recomputed exactly with the
// moved voxels as centres at their centroid cells (c3_hlac.cpp:349-377), normalised, its
// exist gate rewritten, and a newly non-empty one appended to the row list.
struct PointFixup {
  int nf;
  const uint32_t* grid[kMaxBatch];    // canvas grids
  const VoxMoved* moved;              // [nf][kVbMovedCap]
  const uint32_t* xcnt;               // [nf][4]
  const VoxFrameRec* info;            // [nf] (min_b / max_b: the frame's grid)
  int C[3];                           // canvas dims
  const int16_t* axmap;               // canvas coordinate -> subdivision (-1: no centre)
  const int32_t* segs;                // [3][seg_stride][3] start, len, subdivision
  int ns0, ns1, seg_stride;
  int sbx, sby;
  int variant, thr[3];
  const uint32_t* lut;
  float* feat;
  int32_t* exist;
  int32_t* rows;
  uint32_t* tf;                       // per frame: [2] reserved | [2] work counters | stamps
  int64_t s_feat, s_h, s_tf;
  uint32_t epoch;
  int lmax[3];                        // the largest tile (LDS of the recompute)
};
hipError_t launch_point_fixup(const PointFixup& a, hipStream_t s);
bool point_fixup_fits(const int lmax[3]);  // the recompute's LDS (tile halo, list, operands) fits a CU
hipError_t launch_vox_batch(const VoxBatchArgs& a, hipStream_t s);
// the same in two parts: the accumulate (with the clear of the set's previous words), and the
// chain that reads the accumulators (reduce, scatter, exact pass); only the chain reads the
// batch's C3 launch (tile stamps, work lists)
hipError_t launch_vox_batch_accum(const VoxBatchArgs& a, hipStream_t s);
hipError_t launch_vox_batch_post(const VoxBatchArgs& a, hipStream_t s);

struct C3Launch {
  const uint32_t* grid[kMaxBatch];  // one grid per frame of the batch
  int nframes;
  // per-frame buffers: frame f at base + f * stride
  int64_t s_feat, s_h, s_acc, s_tf, s_work;
  uint32_t* tf;           // [2] reserved | [2] work counters | [ntiles] epoch stamps
  int gx, gy, gz;
  const int32_t* segs;  // [3][nseg_max][3] = start, len, subdiv
  int nseg[3];
  int seg_stride;
  int sbx, sby;
  int lmax[3];  // max segment length per axis (LDS tile dims)
  int thr[3];
  int variant;
  int atomic;
  const uint32_t* lut;  // 256 packed entries
  float* feat;
  int32_t* exist;
  unsigned long long* acc64;
  const int16_t* axmap;   // per-axis centre coordinate -> segment index (-1 = none)
  // the y and z maps in closed form, when they are: c >= off ? (c - off) / S : -1
  // (ar_s = S, 0 = use the maps; the division by S as a multiply-high by ar_magic)
  int ar_s = 0, ar_oy = 0, ar_oz = 0;
  uint32_t ar_magic = 0;
  int32_t* work;          // ntiles: non-empty tiles (pass 1 output)
  int32_t* rows;          // direct mode: non-empty subdivision list output (nullable)
  uint32_t epoch;
  int zero_empty;
  int zero_feat;          // zero role also zero-fills feature rows (else exist only)
  int64_t ntiles;
  long long* prof;  // diagnostics (C3H_PROF)
  int debug;
  uint32_t* dense = nullptr;  // stand-alone large grids: the density probe's verdict word
  // fp16 search precision on large grids: the dense MFMA body writes the feature rows as
  // f16 (row stride f16s halves) and sets *feat16_flag; the f32 rows are then not written
  _Float16* feat16 = nullptr;
  uint32_t* feat16_flag = nullptr;
  int f16s = 0;
  // the grid of the last c3h_voxelize (round 6): its scatter listed every occupied voxel's
  // grid index (segment b of vl_seg positions at vl_words + b * vl_seg, vl_counts[b *
  // vl_count_stride] of them), so the tiles are stamped from that list and the occupancy
  // stream over the whole grid is skipped; nullptr: stream the grid
  const uint32_t* vl_words = nullptr;
  const int32_t* vl_counts = nullptr;
  int vl_nseg = 0, vl_seg = 0, vl_count_stride = 0;
};

int64_t c3hlac_grid(const C3Launch& a);  // persistent grid of the tile kernel
hipError_t launch_c3hlac(const C3Launch& a, hipStream_t s);
// colour.hip: per-channel 256-bin histograms of the occupied voxels (adds into out[768])
hipError_t launch_colour_hist(const uint32_t* grid, int64_t nvox, unsigned long long* out, hipStream_t s);
// voxels whose centroid cells differ from their own (exact 64-bit sums, before finalize)
hipError_t launch_offcell_delta(const int32_t* rec, int nrec, const C3Launch& l, int hist1, const int off[3],
                                const int sb[3], float inv_s, hipStream_t s);
hipError_t launch_c3_finalize(const unsigned long long* acc64, int64_t hist_num, int variant,
                              float* feat, int32_t* exist, int nframes, hipStream_t s);
// radius-search grid over a point cloud (rsd.hip): cells of `cell` metres from origin,
// the points sorted by cell, per cell its [cstart, cend) range in `sorted`
struct NbrGrid {
  const float4* pts;
  int64_t n;
  float origin[3];
  float cell, inv_cell;
  int dim[3];
  const uint32_t* sorted;
  const uint32_t* cstart;
  const uint32_t* cend;
};
struct GrsdArgs {
  const float4* cent;     // downsampled centroids, leaf-layout order
  int64_t nc;
  const int32_t* layout;  // leaf layout (-1 empty)
  const int32_t* types;   // per centroid
  int32_t* trans;         // hist_num x 6 x 6
  int div_b[3], min_b[3], off[3], sb[3];
  float leaf, inv_leaf, inv_s;
  int hist1;              // one histogram for the whole cloud
};
hipError_t nbr_build(NbrGrid& g, uint32_t* keys, uint32_t* keys2, uint32_t* idx, uint32_t* idx2, void* tmp,
                     size_t* tmp_bytes, hipStream_t s);
hipError_t launch_normals(const NbrGrid& g, float radius, const float vp[3], float4* out, hipStream_t s);
hipError_t launch_rsd(const NbrGrid& g, const float4* nrm, const float4* cent, int64_t nc, float max_dist,
                      float2* radii, int32_t* types, hipStream_t s);
hipError_t launch_grsd(const GrsdArgs& a, hipStream_t s);
hipError_t launch_grsd_feat(const int32_t* trans, int64_t H, float norm, float* out, int stride, hipStream_t s);
hipError_t launch_vosch_concat(const float* grsd, const float* c3, const int32_t* exist, int64_t H, float* out,
                               hipStream_t s);
// sensor_msgs/PointCloud2 bytes -> n x float4 (x, y, z, rgb bits) (ingest.hip)
hipError_t launch_pc2_convert(const void* data, uint32_t height, uint32_t width, uint32_t point_step,
                              uint32_t row_step, const int32_t off[4], int big, float* out, hipStream_t s);
hipError_t launch_exist_rule(const float* feat, int64_t H, int dim, int rule, int32_t* exist, hipStream_t s);

// rows/nrows (device): compress only the listed rows (sparse mode), else all H rows
hipError_t launch_compress(const float* feat, int64_t H, int F, const float* axis_pt, int D,
                           int Dpad, const float* fmax, int fmax_len, float* G,
                           const int32_t* rows, const uint32_t* nrows, const int32_t* exist,
                           hipStream_t s);
// dst[h][:] = exist[h] ? src[h][:] : 0 (readback of buffers whose empty rows are stale)
hipError_t launch_masked_rows(const float* src, const int32_t* exist, int64_t H, int W, float* dst,
                              hipStream_t s);

struct ScoreLaunch {
  const float* G;
  const int32_t* exist;
  int D;
  int xn, yn, zn;
  int xr, yr, zr;
  int xe, ye, ze;
  int thr;
  const float* axis_q;  // M x r x D (generic path)
  const float* qt;      // D x Opad transposed basis (fast path)
  int M, r, Opad;
  double* scores;       // M x P for this mode
  ScorePartial* partials;  // per-block per-model best (nullable)
  int64_t order_base;
};
hipError_t launch_score(const ScoreLaunch& a, hipStream_t s);
bool score_fast_ok(int D, int r);  // the sparse list path applies
int64_t score_blocks(const ScoreLaunch& a);

// sparse search (fast path): gate every position of every mode, project the list
struct ModeGeom {
  int64_t offset;  // into scores (M x P block)
  int64_t P;
  int xe, ye, xr, yr, zr;
  int mode;        // SearchMode id
};
struct SparseSearch {
  const float* G;
  const int32_t* exist;
  int D, xn, yn, zn, thr;
  const float* qt;        // D x Opad (row stride), zero-padded past M*r
  int M, r, Opad;
  int mpg;                // models per workgroup (whole models, mpg*r <= 64)
  int group_loop;         // 1: a workgroup runs every model group over one box-sum pass (tick)
  double* scores;
  ModeGeom md[6];
  int nmodes;
  int64_t pstart[7];      // prefix of P over modes
  int64_t order_base[6];  // mode index << 40
  long long* list;        // gate list entries (mode << 40 | position)
  uint32_t* cnt;          // [2] list counters by epoch parity
  uint32_t epoch;
  int nframes;             // frames of the batch (launch z / y index)
  int64_t s_G, s_exist, s_scores, s_list, s_cnt, s_partials, s_lists;  // per-frame strides
  c3h_det* outs[kMaxBatch];  // per-frame copy of the lists after the update (nullable)
  ScorePartial* partials;  // per block per model (nullable)
  uint32_t* done;          // [2] finished-workgroup counters by epoch parity
  c3h_det* lists;          // rank 1 fused replay: M lists (nullable = no fused replay)
  int clean;               // apply a pending cleanMax first
  long long* prof;         // diagnostics (C3H_PROF): [blocks][8]
  float* gbox = nullptr;   // large grids: box-summed G rows of every position (pstart order)
  int64_t s_gbox = 0;
  int score_mfma = 0;      // project on the matrix cores (score_mfma_kernel; needs gbox, nframes 1)
  int skip_empty = 1;      // box sums skip rows with exist 0 (C3 extracts: exist 0 <=> no centre voxel)
  const _Float16* qt16 = nullptr;  // fp16 search precision: the basis as f16, [Opad][16 * Kq16]
  int Kq16 = 0;                    // 16-wide k steps (D rounded up to 16, / 16)
  // canvas frames (c3h_run_point_frames): per frame its own subdivision counts; a box
  // position passes only when it lies inside them (search.cpp:218-317 over the frame's
  // subdiv_b), so the canvas' extra empty subdivisions add no position
  const int32_t* lim = nullptr;    // [frame][4] (nullable)
  // the score buffers hold the previous search of this layout: a gated-out position whose
  // model-0 score is already -1 has -1 for every model (writers always fill all models of
  // a position), so the gate rewrites only positions that passed last time
  int sparse_scores = 0;
};
bool score_mfma_ok(int D);  // D fits score_mfma_kernel
// sparse compress fused into the gate launch (nullable in launch_sparse_search)
struct SparseCompress {
  const float* feat;
  const float* PT;
  const float* fmax;
  float* G;
  const int32_t* rows;
  const uint32_t* nrows;
  int F, D, Dpad, fmax_len;
  int64_t H;
  int64_t s_feat, s_G, s_rows, s_nrows;  // per-frame strides
  const _Float16* PT16 = nullptr;         // fp16 search precision: f16 axis, 128 x Fp16
  int Fp16 = 0;
  const _Float16* feat16 = nullptr;       // f16 feature rows (stride f16s) when *feat16_flag
  const uint32_t* feat16_flag = nullptr;
  int f16s = 0;
};
bool compress_rows_ok(int F, int Dpad);
constexpr int64_t kBoxsumRows = 65536;  // subdivisions from which the search precomputes box sums
constexpr int64_t kCompressMfmaRows = 65536;  // ... and compresses on the matrix cores
hipError_t launch_sparse_search(const SparseSearch& a, const SparseCompress* sc, hipStream_t s);
int64_t sparse_score_blocks(const SparseSearch& a);

struct ReplayMode {
  int64_t offset;  // into scores (M x P block)
  int64_t P;
  int xe, ye;
  int mode;
};
struct ReplayModes {
  ReplayMode m[6];
  int n;
};
hipError_t launch_replay(const double* scores, const ReplayModes& modes, int M, int rank,
                         int r1, int r2, int r3, int clean, c3h_det* lists, c3h_det* out2,
                         hipStream_t s);

hipError_t launch_clean_lists(c3h_det* lists, int n, hipStream_t s);

// one pipeline tick of c3h_run_frames (pipeline.hip): every role nullable
struct TickParts {
  const C3Launch* occ = nullptr;        // batch t: occupancy stream
  const C3Launch* tile = nullptr;       // batch t-1: C3 tile pass
  const SparseSearch* gate = nullptr;   // batch t-2: exist gate ...
  const SparseCompress* comp = nullptr; //   ... + sparse compress
  const SparseSearch* score = nullptr;  // batch t-3: list scoring + rank-1 argmax
  DevBuf<long long>* prof = nullptr;    // diagnostics builds: the context's timestamp buffer
};
bool tick_ok(const C3Launch& l);  // the C3 launch fits the tick's roles
hipError_t launch_tick(const TickParts& p, hipStream_t s);
size_t c3hlac_lds_bytes(int tw_max, int list_max);
int64_t leaf_layout_blocks(int64_t nvox);

}  // namespace c3h

struct c3h_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  std::string err;

  // frame lanes of c3h_run_frames: child contexts on their own streams (frames are
  // independent, so K frames are in flight at once); children time into the parent
  c3h_ctx* parent = nullptr;
  std::vector<c3h_ctx*> lanes;
  std::vector<hipEvent_t> lane_ev;
  hipEvent_t fork_ev = nullptr;
  int nlanes = 3;
  int nbatch = 32;                  // frames per launch in c3h_run_frames
  bool pipeline = true;             // c3h_run_frames: pipelined tick launches (else lanes)
  // host copy of the search setup, replayed into the lanes
  uint64_t setup_version = 0;
  std::vector<float> h_axis_p, h_var, h_axis_q, h_fmax;

  // voxel grid
  bool have_grid = false;
  c3h_grid_info info{};
  c3h::DevBuf<uint32_t> grid;       // owned packed grid
  const uint32_t* grid_ptr = nullptr;  // the grid in use (owned or bound)
  c3h::DevBuf<float> pts;           // staging copy of host points
  c3h::DevBuf<uint32_t> raw;        // staging copy of host PointCloud2 bytes
  c3h::DevBuf<float> dsbuf;         // host readback staging of the downsampled cloud
  // normals / RSD / GRSD (rsd.hip): radius-search grid of the last voxelize's points
  c3h::DevBuf<float4> normals;
  bool normals_valid = false;
  c3h::NbrGrid nbr{};
  c3h::DevBuf<uint32_t> nkeys, nkeys2, nidx, nidx2, ncstart, ncend;
  c3h::DevBuf<uint8_t> ntmp;
  c3h::DevBuf<float4> dsamp;        // downsampled centroids (leaf-layout order)
  c3h::DevBuf<float2> rsd_radii;
  c3h::DevBuf<int32_t> rsd_types, grsd_trans;
  c3h::DevBuf<float> grsd_feat, vosch_feat;
  int64_t rsd_n = 0;                // centroids with valid radii / types
  // voxeliser state (voxelize.hip): toroidal accumulators, entry / grid-word lists by
  // epoch parity, counters; the grid words the previous frame wrote are cleared by the next
  c3h::DevBuf<ulonglong2> vacc;
  c3h::DevBuf<uint32_t> vmg;
  c3h::DevBuf<uint32_t> vtpos, vlists, vlcnt, vcnt;
  c3h::DevBuf<int32_t> vpart;
  int vtb[3] = {7, 7, 7};           // toroidal dims (log2 per axis); they only grow
  int64_t vtor = 0;                 // cells of the allocated accumulators (0: none)
  uint64_t vlcap = 0;
  int vpar = 0, vblk_cap = 0;
  int vblk_prev = 0;                // accum blocks of the previous frame (its lists to clear)
  bool vgrid_tracked = false;       // grid buffer is zero outside the previous frame's list
  c3h::VoxArgs vargs{};             // the last voxelize (exact centroid pass, downsampled)
  int64_t vns = 0;                  // voxels of the last voxelize
  // exact centroid pass: per-voxel counts / offsets / cursors, point buckets, centroids,
  // off-cell records {idx, neighbour-base cell xyz, subdivision cell xyz, 0}
  c3h::DevBuf<uint32_t> vcounts, voffs, vcur, vbucket;
  c3h::DevBuf<float4> vcent;
  c3h::DevBuf<int32_t> voffcell;
  bool vcent_valid = false;
  int64_t n_offcell = 0;
  c3h::DevBuf<uint32_t> scratch;    // minmax / counters
  c3h::DevBuf<uint32_t> tmp_u32;    // leaf-layout block sums
  c3h::DevBuf<int32_t> tmp_i32;     // leaf layout for host copies
  uint32_t* h_small = nullptr;      // pinned host scratch (64 words)
  c3h::VoxFrameRec* h_recs = nullptr;  // pinned: the frame records a c3h_run_point_frames call reads back
  size_t h_recs_n = 0;
  bool table_valid = false;         // hash table matches the grid (voxelize path)

  // features
  bool have_feat = false;
  c3h_extract_params last{};
  int64_t hist_num = 0;
  int32_t subdiv_b[3] = {0, 0, 0};
  int feat_dim = 0;
  c3h::DevBuf<float> feat;
  c3h::DevBuf<int32_t> exist;
  c3h::DevBuf<unsigned long long> acc64;
  c3h::DevBuf<int32_t> segs;        // per-axis tile segment tables
  c3h::DevBuf<int16_t> axmap;       // per-axis coordinate -> segment (pass-1 tile lookup)
  std::vector<int16_t> h_axmap;
  c3h::DevBuf<uint32_t> tileflags;  // [2] reserved | [2] work counters | [ntiles] stamps
  c3h::DevBuf<int32_t> work;        // non-empty tiles of the last extract
  uint32_t tile_epoch = 0;
  int cap_h2d = 0;  // tables / stamp resets extract_frames enqueued (counts; points-in ordering)
  int64_t tf_stride = -1;           // tile-stamp layout the counters were zeroed for
  int tf_frames = 0;
  int nframes_feat = 1;             // frames of the last extract (frame 0 = the API view)
  c3h::DevBuf<int32_t> rows;        // non-empty subdivisions of the last extract (direct mode)
  bool rows_valid = false;          // rows/epoch describe the current features
  bool g_sparse = false;            // G holds only the listed rows (others stale)
  bool feat_sparse = false;         // feature rows of empty subdivisions are stale (exist == 0)
  c3h::DevBuf<long long> glist;     // sparse search: gate list
  c3h::DevBuf<float> gbox;          // large grids: box sums of G per position (P_total x D)
  c3h::DevBuf<uint32_t> gcnt;       // [2] gate-list counters by search epoch parity
  uint32_t search_epoch = 0;
  int gcnt_frames = 0;
  c3h::DevBuf<long long> prof;      // diagnostics (C3H_PROF)
  c3h::DevBuf<unsigned long long> chist;  // colour histograms (c3h_color_histogram): 3 x 256

  std::vector<int32_t> h_segs;      // host copy (kept alive for the async upload)
  c3h::DevBuf<uint32_t> lut;        // 256 packed (sin | cos<<8), two variants
  bool lut_ready = false;

  // search
  bool have_setup = false;
  int D = 0, F = 0, M = 0, r = 0, Dpad = 0;
  // exist 0 implies an all-zero feature row (C3 extracts: every centre voxel adds >= 1 to
  // the exist value); GRSD / VOSCH / caller features do not promise it (a row of a few
  // GRSD transitions has exist 0), so their box sums add every row as searchPart does
  bool exist_gates_rows = false;
  int D_user = 0;  // the caller's D (D is rounded up to a multiple of 4 with zero axes)
  bool compress = true;
  c3h::DevBuf<float> axis_pt;       // F x Dpad (transposed, whitened)
  c3h::DevBuf<_Float16> axis_pt16;  // 128 x Fp16 f16 copy (column-major) for the fp16 compress
  int Fp16 = 0;
  bool prec16 = false;              // c3h_set_search_precision: fp16 matrix-core compress
  c3h::DevBuf<_Float16> feat16;     // f16 feature rows of the last large dense extract (prec16)
  c3h::DevBuf<uint32_t> feat16_flag;
  bool feat16_pending = false;      // the last extract may have written f16 rows only
  int feat16_s = 0;                 // their row stride (halves)
  int score_engine = 0;             // c3h_set_score_engine: 0 auto, 1 VALU, 2 matrix cores
  c3h::DevBuf<_Float16> qt16;       // f16 basis for the fp16 matrix-core projection
  int Kq16 = 0;
  c3h::DevBuf<float> axis_q;        // M x r x D
  c3h::DevBuf<float> fmax;
  int fmax_len = 0;
  c3h::DevBuf<float> G;             // hist_num x D compressed features
  bool g_valid = false;
  c3h::DevBuf<double> scores;
  int64_t scores_n = 0;
  // layout of the score buffers' last search (modes' offsets and sizes, M, frames, buffer):
  // an equal layout lets the gate skip the -1 fill of positions already gated out
  // layout of the last search whose gate was enqueued on `scores` (empty: unknown); a search
  // of the same layout writes -1 only where that one had not gated the position out already
  std::vector<int64_t> scores_layout;
  std::vector<int64_t> cap_layout;  // a captured (pipelined) search's layout, until its gate runs
  c3h::DevBuf<float> qt;            // D x Opad transposed model basis (fast score path)
  int Opad = 0;
  c3h::DevBuf<c3h::ScorePartial> partials;
  bool pending_clean = false;       // cleanMax requested while the device lists are current
  int rank = 1;
  c3h::SearchLists lists;
  std::vector<c3h_det> h_lists;     // host staging of the lists
  c3h_det* h_dl = nullptr;  // pinned: the lists a search reads back (one async copy + one sync)
  size_t h_dl_n = 0;
  c3h::DevBuf<c3h_det> d_lists;
  bool lists_host_valid = true;     // host lists are current
  bool lists_dev_valid = false;     // device lists are current
  int32_t last_range[3] = {0, 0, 0};

  c3h::Timer timer;

  // capture mode (c3h_run_frames pipeline): extract/search record their launches here
  // instead of enqueueing them
  bool capture = false;
  bool cap_c3_valid = false, cap_search_valid = false, cap_sparse_g = false, cap_argmax = false;
  c3h::C3Launch cap_c3{};
  c3h::SparseSearch cap_q{};
  c3h::SparseCompress cap_sc{};

  // the software pipeline of c3h_run_frames / c3h_stream_frames: batches whose later
  // stages are still to run, each tagged with the tick role it runs next (1 tile,
  // 2 compress+gate, 3 score); the buffer set of batch number s is s % 4 (0 = this
  // context, k = lanes[k-1]); `key` identifies the stream's geometry and parameters
  struct PipeBatch {
    c3h::C3Launch l;
    c3h::SparseSearch q;
    c3h::SparseCompress sc;
    int nf;
    int age;
    bool stamped = false;  // tile stamps already set (points-in scatter): no occupancy role
    c3h_ctx* set = nullptr;       // the buffer set (context) the batch was captured on
    std::vector<int64_t> layout;  // its score-array layout, recorded there once its gate is enqueued
    bool fix = false;             // points-in batch: the off-cell fixup runs after its tile role
    c3h::PointFixup fx{};
  };
  struct PipeKey {
    int32_t div_b[3], min_b[3];
    float leaf;
    c3h_extract_params p;
    int32_t range[3], thr, rotate, batch, rank;
    uint64_t setup_version;
  };
  // points-in batches (c3h_run_point_frames).  Per buffer set: the canvas grids of its frame
  // slots, the words its last batch wrote (cleared by the next batch on the set), the
  // partial records and the gate limits.  Shared (the calling context): the toroidal
  // accumulators, the voxel lists, host-point staging, the frames' records.
  c3h::DevBuf<uint32_t> pb_grid, pb_wlist;
  c3h::DevBuf<int32_t> pb_part, pb_lim;
  c3h::DevBuf<c3h::VoxFlag> pb_flags;    // the exact pass of this set's batch
  c3h::DevBuf<uint32_t> pb_bucket, pb_xcnt;
  c3h::DevBuf<uint32_t> dense_flag;  // density probe of large stand-alone extracts
  c3h::DevBuf<c3h::VoxMoved> pb_moved;
  int64_t pb_cvox = 0;             // canvas voxels per slot the set's buffers hold
  int pb_slots = 0;
  int pb_prev_nf = 0, pb_prev_total = 0;
  std::vector<int> pb_prev_blk0;
  c3h::DevBuf<ulonglong2> pb_acc;
  c3h::DevBuf<uint32_t> pb_accM, pb_vlist, pb_fcnt;
  int64_t pb_acc_vox = 0;
  int pb_acc_slots = 0;
  c3h::DevBuf<float> pb_stage;
  c3h::DevBuf<c3h::VoxFrameRec> pb_info;
  // the batched voxeliser runs on its own stream, one batch ahead of the tick that consumes
  // it (events: a batch's voxels are done / the tick that last read a buffer set is done)
  hipStream_t pb_vstream = nullptr;
  // c3h_voxelize of host frames: the chunked H2D's stream, its start and per-chunk events
  hipStream_t vcopy = nullptr;
  hipEvent_t vcopy_start = nullptr;
  std::vector<hipEvent_t> vcopy_ev;
  hipEvent_t pb_vox_ev = nullptr, pb_tick_ev[4] = {nullptr, nullptr, nullptr, nullptr};

  std::vector<PipeBatch> pipe;   // in flight, oldest first
  uint64_t pipe_seq = 0;
  PipeKey pipe_key{};
  int pipe_nm = 0;
  bool pipe_busy = false;        // inside a pipeline call (set contexts are being prepared)
};

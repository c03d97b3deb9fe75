// c3hlac_mfma.h -- dense C3-HLAC tiles on the i8 matrix cores (v_mfma_i32_16x16x64_i8).
//
// Same result as the dot4 tile body (c3hlac_dev.h), for tiles whose centre voxels are
// mostly occupied (config 5: 512^3 at 100 %), where compacting occupied voxels saves
// nothing.  Every bin is an exact integer correlation over the tile's centre voxels v
//   C_k[c][n] = sum_v X_c(v) * Y_n(v + r_k)
// of 12 channels (6 sin/cos LUT colour bytes r,r_,g,g_,b,b_ and 6 binary beta, 1-beta;
// all 0 for empty voxels) with the 13 half-neighbourhood offsets r_k (c3_hlac.cpp:177-202)
// plus k = 13, the centre's own channels (auto products, bin-pair counts).  That is one
// 16 x 16 x K integer GEMM per k with K = centre voxels:
//   A = X (row c = channel, 12 of 16 rows), B_k = Y shifted by r_k (column n = channel).
// u8 channel values are stored offset by -128 (byte ^ 0x80), which i8 holds exactly, and
// the exact sums are recovered with the padding rows / columns: row 15 of A and column 15
// of B are constant 1, so
//   sum a b = C[c][n] + 128 (C[c][15] + C[15][n]) + 128^2 C[15][15]
// elementwise over the K positions: a position that is no centre carries a = 0 (A' = -128,
// whatever B holds there), so the K positions need not all be centres.  C[c][15] is the
// same for every k (A does not move), C[15][15] is the position count.  u32 arithmetic is
// exact (every true sum is < 2^32; |a' b'| <= 2^14 per position).
//
// Mapping: one wave per tile (<= 16 x 16 centres per layer), walking the tile's layers in
// z.  Layer L (z = z0 - 1 + L) is held in LDS as 12 channel planes, each the layer's
// (ly + 2) rows of (lx + 2) bytes (halo included) at a row pitch PW = lx + 2 rounded up to
// 4, packed one after another: a voxel's neighbour at (dx, dy) is dy * PW + dx bytes away.
// A K step is 64 consecutive plane positions (lane group h = lane >> 4 takes 16 of them)
// starting at row 1, so a K step spans row boundaries and only the positions that are
// centres count (a per-tile byte mask plane); S = 10 tiles take 2 K steps per layer where a
// 16-byte row per lane group took 3.  The K origin is 16-byte aligned; PW mod 16 (0, 4, 8,
// 12) is a template parameter, so every fragment is read as aligned dwords (ds_read_b128 /
// b64 / b32 by its alignment) and the dx = +-1 shifts are one v_alignbyte per dword.  Per K
// step: 5 plane rows + the mask, 14 MFMAs.  The next layer's grid words are loaded into
// registers two layers ahead (three layer slots in a ring).  The epilogue corrects and
// scatters the accumulator tiles from registers (the padding lanes' sums by ds_bpermute).
// Round 6: tiles of two-step layers (S <= 10, pitch 12: every interior tile of config 5)
// hold each layer as a voxel-major record image instead of channel planes and read the
// operands back through ds_read_b64_tr_b8 (mf_layer_ksteps_tr): the conversion needs no
// byte transpose, and the dx shifts are immediate address offsets.
#pragma once
#include "c3hlac_dev.h"

namespace c3h {

typedef int mf_v4i __attribute__((ext_vector_type(4)));
constexpr int kMfWaves = kBlock / 64;
constexpr int kMfCh = 12;
constexpr int kMfK = 14;    // 13 offsets + the centre's own channels
constexpr int kMfLoad = 2;  // (row, dword) items per lane of a layer (<= 18 rows x 5 dwords)
#ifndef C3H_MF_TWO
#define C3H_MF_TWO 1  // two-step layers with the lane-group-contiguous position map
#endif
#ifndef C3H_MF_GAP
#define C3H_MF_GAP 16  // diagnostics: 0 = the round-3 plane placement of the two-step layers
#endif
#ifndef C3H_MF_EXP
#define C3H_MF_EXP 0  // diagnostics variants: 1 no K steps, 2 no conversion, 4 no bin epilogue, 8 no layer loads
#endif

__host__ __device__ inline int mf_pitch(int lx) { return (lx + 2 + 3) & ~3; }
// items per lane of a layer for tiles up to lx x ly: (ly + 2) rows x pitch / 4 dwords
__host__ __device__ inline int mf_load_items(int lx, int ly) { return ((ly + 2) * (mf_pitch(lx) >> 2) + 63) / 64; }
// byte of position 0 in a plane: (off0 + PW) % 16 == 0 (the K origin), >= 16 bytes of
// headroom for the dy = -1 reads of the first K step
__host__ __device__ inline int mf_off0(int pw) { return 16 + ((16 - (pw & 15)) & 15); }
__host__ __device__ inline int mf_nks(int lx, int ly, int pw) { return ((ly - 1) * pw + lx + 1 + 63) / 64; }
// LDS banks: a ds_read_b128 serves 16 lanes per cycle, lane (h, n) reading 16 bytes of
// plane n at chunk h.  With the plane stride = 32 mod 256 bytes, the layer slots and the
// wave regions 256-byte aligned and the constant planes (read by lanes n >= 12) at 128 mod
// 256, every lane group's 16 reads hit 16 distinct 4-bank blocks (no conflicts; a stride of
// 192 bytes was 2-way).
__host__ __device__ inline int mf_plane_bytes(int lx, int ly) {
  const int pw = mf_pitch(lx), o = mf_off0(pw), n = mf_nks(lx, ly, pw);
  const int a = o + (ly + 2) * pw, b = o + 2 * pw + 64 * n + 16;
  const int m = a > b ? a : b;
  return ((m - 32 + 255) & ~255) + 32;
}
__host__ __device__ inline int mf_r256(int x) { return (x + 255) & ~255; }
// (+16: the two-step layers put planes 4..11 one 16-byte block further, see mf_layer_ksteps2)
__host__ __device__ inline int mf_slot_stride(int pb) { return mf_r256(kMfCh * pb + 16); }
#ifndef C3H_MF_SLOTS
#define C3H_MF_SLOTS 3  // layer slots per wave (2: layer z + 2 reuses layer z's slot after its K steps)
#endif
constexpr int kMfSlots = C3H_MF_SLOTS;
static_assert(kMfSlots == 2 || kMfSlots == 3, "layer slots");
__host__ __device__ inline int mf_wave_stride(int pb) { return kMfSlots * mf_slot_stride(pb) + mf_r256(pb); }
__host__ __device__ inline int mf_const_bytes(int pb) { return mf_r256(128 + 3 * pb); }
// 3 x 256 channel-byte tables | 128 B | 3 constant planes (0x00, 0x01, 0xff) | per-wave
// regions: 3 layer slots of 12 planes, the centre mask
// 981 epilogue (round 5): every accumulator value is staged in the wave's idle plane
// slots at (k, row c, column n) -- stage index k * 144 + ((c >> 2) * 12 + n) * 4 + (c & 3),
// the 12 zero-order sums at 14 * 144 + c -- and the row is gathered bin by bin through a
// per-workgroup source table (981 u16 after the wave regions)
constexpr int kMfStage = 14 * 144 + 12;  // floats per wave
constexpr int kMfSrcBytes = 2048;
static_assert(kMfSlots == 3, "the 981 staging needs the three layer slots (>= 10,752 bytes)");
__host__ __device__ inline size_t mf_lds_bytes(int pb) {
  return 3072 + (size_t)mf_const_bytes(pb) + (size_t)kMfWaves * mf_wave_stride(pb) + kMfSrcBytes;
}
// the tables and the 128-byte gap are the kernel's static LDS; the rest is dynamic
constexpr int kMfStaticWords = 800;
__host__ __device__ inline size_t mf_dyn_lds_bytes(int pb) { return mf_lds_bytes(pb) - 4 * kMfStaticWords; }
static_assert(4 * kMfStage <= 3 * 3584, "stage fits the layer slots of the smallest plane (288 B)");

// channel plane of (type t: 0 colour LUT / 1 binary, reference channel c in 0..5): the
// planes hold per colour col the bytes {sin, cos, beta, 1 - beta} (4 col + s)
__host__ __device__ inline int mf_plane(int t, int c) { return 4 * (c >> 1) + 2 * t + (c & 1); }

__device__ __forceinline__ void mf_compiler_fence() { __asm__ volatile("" ::: "memory"); }

typedef uint32_t mf_u4 __attribute__((ext_vector_type(4)));
constexpr int mf_fdiv16(int x) { return x >= 0 ? x / 16 : -((15 - x) / 16); }

// The 16-byte blocks of a plane row holding the bytes at DYR + dx .. + 15 for dx in
// [DXLO, DXHI] (DYR = dy * (PW mod 16), compile time), read from the row's 16-byte aligned
// base as whole ds_read_b128 blocks, and its dx fragments (v_alignbyte for dx = +-1)
template <int DYR, int DXLO, int DXHI>
struct MfRow {
  static constexpr int B0 = mf_fdiv16(DYR + DXLO), NB = mf_fdiv16(DYR + DXHI + 15) - B0 + 1;
  uint32_t w[4 * NB];
  __device__ __forceinline__ void load(const uint8_t* row) {
    const uint8_t* p = static_cast<const uint8_t*>(__builtin_assume_aligned(row, 16));
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      mf_u4 v = *reinterpret_cast<const mf_u4*>(p + 16 * (B0 + b));
      __asm__("" : "+v"(v));  // keep the whole block: a narrowed ds_read_b32 bank-conflicts
      w[4 * b] = v.x; w[4 * b + 1] = v.y; w[4 * b + 2] = v.z; w[4 * b + 3] = v.w;
    }
  }
  template <int DX>
  __device__ __forceinline__ mf_v4i frag() const {
    constexpr int e = DYR + DX - 16 * B0, d = e >> 2, sh = e & 3;
    mf_v4i f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      f[i] = sh ? (int)__builtin_amdgcn_alignbyte(w[d + i + 1], w[d + i], sh) : (int)w[d + i];
    return f;
  }
};

constexpr int kMfMaxKs = 5;  // K steps per layer of a 16 x 16 tile (PW = 20)

// The K steps of one layer.  pp / pc / pm: this lane's dz = -1 plane, dz = 0 plane and mask
// plane at the K origin (byte off0 + PW, 16-byte aligned); pw16 = PW - R.  The six row
// pointers are formed once per layer; the K steps are unrolled, so their offsets (64 ks) are
// instruction immediates.
template <int R>
__device__ __forceinline__ void mf_layer_ksteps(const uint8_t* pp, const uint8_t* pc, const uint8_t* pm, int pw16,
                                                int nks, int h4, mf_v4i (&acc)[kMfK]) {
  const int o = 16 * h4;
  const uint8_t* r_c0 = pc + o;          // dz = 0, dy = 0
  const uint8_t* r_cm = pc + o - pw16;   // dz = 0, dy = -1
  const uint8_t* r_pm = pp + o - pw16;   // dz = -1, dy = -1
  const uint8_t* r_p0 = pp + o;          // dz = -1, dy = 0
  const uint8_t* r_pp = pp + o + pw16;   // dz = -1, dy = +1
  const uint8_t* r_m = pm + o;
#pragma unroll
  for (int ks = 0; ks < kMfMaxKs; ++ks) {
    if (ks >= nks) break;
    const int ko = 64 * ks;
    // dz = 0: row 0 (the centres and dx = -1), row -1
    MfRow<0, -1, 0> c0;
    MfRow<-R, -1, 1> cm;
    c0.load(r_c0 + ko);
    cm.load(r_cm + ko);
    const mf_u4 m = *reinterpret_cast<const mf_u4*>(__builtin_assume_aligned(r_m + ko, 16));
    const mf_v4i a0 = c0.frag<0>();
    mf_v4i A;
#pragma unroll
    for (int i = 0; i < 4; ++i) A[i] = (int)(((uint32_t)a0[i] & m[i]) | (0x80808080u & ~m[i]));
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, A, acc[13], 0, 0, 0);                  // own channels
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, c0.frag<-1>(), acc[12], 0, 0, 0);  // (-1, 0, 0)
    acc[9] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, cm.template frag<-1>(), acc[9], 0, 0, 0);    // (dx, -1, 0)
    acc[10] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, cm.template frag<0>(), acc[10], 0, 0, 0);
    acc[11] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, cm.template frag<1>(), acc[11], 0, 0, 0);
    // dz = -1, rows dy = -1, 0, +1: k = 3 (dx + 1) + (dy + 1)
    {
      MfRow<-R, -1, 1> r;
      r.load(r_pm + ko);
      acc[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<-1>(), acc[0], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<0>(), acc[3], 0, 0, 0);
      acc[6] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<1>(), acc[6], 0, 0, 0);
    }
    {
      MfRow<0, -1, 1> r;
      r.load(r_p0 + ko);
      acc[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<-1>(), acc[1], 0, 0, 0);
      acc[4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<0>(), acc[4], 0, 0, 0);
      acc[7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<1>(), acc[7], 0, 0, 0);
    }
    {
      MfRow<R, -1, 1> r;
      r.load(r_pp + ko);
      acc[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<-1>(), acc[2], 0, 0, 0);
      acc[5] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<0>(), acc[5], 0, 0, 0);
      acc[8] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, r.template frag<1>(), acc[8], 0, 0, 0);
    }
  }
}

// Layers of exactly two K steps (S <= 10 tiles: pitch 12, 12 rows -> 128 positions): lane
// group h takes the 32 consecutive positions 32 h .. 32 h + 31 over both steps (K step ks
// gets 32 h + 16 ks + i; the position -> (step, lane group, byte) map is a bijection and A,
// B and the mask use the same one, so the integer sums are unchanged).  A plane row then
// costs NB = 3-4 ds_read_b128 for both steps instead of 2 x 2-3: 16 instead of 22 reads
// per layer, and the centre mask (the same plane for every layer) stays in registers.
// Banks: lane (h, n) reads plane n at 32 h, so with planes at a 288-byte stride (18 blocks
// of 16 B) the 4-bank block of every lane is even and a ds_read_b128 lane group (lanes
// {0-3, 12-15, 20-27} = (h 0, n 0-3 / 12-15), (h 1, n 4-11), ...) met its own blocks twice
// (2-way, every read).  Planes 4..11 then sit one block further (odd blocks): the 12 real
// lanes of each group hit 12 distinct blocks and the constant planes (blocks 8, 10) the
// rest.  The one-step layout (16 h) is conflict-free without the shift.
template <int DYR, int DXLO, int DXHI>
struct MfRow2 {
  static constexpr int B0 = mf_fdiv16(DYR + DXLO), NB = mf_fdiv16(DYR + DXHI + 31) - B0 + 1;
  uint32_t w[4 * NB];
  mf_u4 q[NB];
  __device__ __forceinline__ void load(const uint8_t* row) {
    const uint8_t* p = static_cast<const uint8_t*>(__builtin_assume_aligned(row, 16));
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      mf_u4 v = *reinterpret_cast<const mf_u4*>(p + 16 * (B0 + b));
      __asm__("" : "+v"(v));  // keep the whole block: a narrowed ds_read_b32 bank-conflicts
      w[4 * b] = v.x; w[4 * b + 1] = v.y; w[4 * b + 2] = v.z; w[4 * b + 3] = v.w;
    }
  }
  // prefetch: issue() the reads, pin() where the row is first used -- the whole-block
  // barrier then sits after the work issued in between, which hides the LDS latency
  __device__ __forceinline__ void issue(const uint8_t* row) {
    const uint8_t* p = static_cast<const uint8_t*>(__builtin_assume_aligned(row, 16));
#pragma unroll
    for (int b = 0; b < NB; ++b) q[b] = *reinterpret_cast<const mf_u4*>(p + 16 * (B0 + b));
  }
  __device__ __forceinline__ void pin() {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      mf_u4 v = q[b];
      __asm__("" : "+v"(v));
      w[4 * b] = v.x; w[4 * b + 1] = v.y; w[4 * b + 2] = v.z; w[4 * b + 3] = v.w;
    }
  }
  template <int DX, int KS>
  __device__ __forceinline__ mf_v4i frag() const {
    constexpr int e = DYR + DX + 16 * KS - 16 * B0, d = e >> 2, sh = e & 3;
    mf_v4i f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      f[i] = sh ? (int)__builtin_amdgcn_alignbyte(w[d + i + 1], w[d + i], sh) : (int)w[d + i];
    return f;
  }
};

#ifndef C3H_MF_PREFETCH
#define C3H_MF_PREFETCH 1  // two-step layers: each plane row's reads issued one row ahead
#endif
#ifndef C3H_MF_ASHIFT
#define C3H_MF_ASHIFT 1  // two-step layers: the dx shifts on the centre operand (round 5)
#endif

// Two-step layers with the x shifts moved to the centre operand (round 5).  An offset
// (dx, R) pairs the centre at position v with the neighbour at v + dx + R; written over
// K = v + dx, that is A_s[K] = Xm(K + s) with s = -dx against the UNSHIFTED neighbour row
// B[K] = Y(K + R).  The three dx of a row then share one B fragment, and only the masked
// centre row is shifted: per K step two 4-dword v_alignbyte sets (A_{+1}, A_{-1}) instead
// of two per neighbour row, and the centre mask is applied once, to the 10 dwords a lane
// group's positions and their +-1 bytes span (mk: the tile's mask words, once per tile).
// Each A_s still visits every centre exactly once: centres lie at K positions 1 ..
// (ly - 1) PW + lx <= 118 of 0 .. 127, so A_{+1} (positions 1 .. 128) and A_{-1} (-1 ..
// 126) cover them, and the positions a shift moves in or out (-1, 0, 127, 128) are
// never centres: every A_s has the same row sums (the epilogue's rs) and
// sum (A'+128)(B'+128) over K is the exact sum over centres, whatever B holds elsewhere.
template <int R>
__device__ __forceinline__ void mf_layer_ksteps2s(const uint8_t* pp, const uint8_t* pc, const uint32_t (&mk)[10],
                                                  int pw16, int h4, mf_v4i (&acc)[kMfK]) {
  const int o = 32 * h4;
  MfRow2<0, -1, 1> c0;   // dz = 0, dy = 0: bytes -16 .. +48 around the lane group's 32
  MfRow2<-R, 0, 0> cm;   // dz = 0, dy = -1 (k = 9 + dx + 1)
  c0.issue(pc + o);
  cm.issue(pc + o - pw16);
  c0.pin();
  // masked centre words am[j] = bytes 32 h + 4 (j - 1) .. + 3 (c0.w index j + 3: B0 = -1)
  uint32_t am[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) am[j] = (c0.w[j + 3] & mk[j]) | (0x80808080u & ~mk[j]);
  mf_v4i A[3][2];  // [s + 1][ks]: A_s of K step ks
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * ks + i + 1;
      A[1][ks][i] = (int)am[j];
      A[2][ks][i] = (int)__builtin_amdgcn_alignbyte(am[j + 1], am[j], 1);  // s = +1
      A[0][ks][i] = (int)__builtin_amdgcn_alignbyte(am[j], am[j - 1], 3);  // s = -1
    }
  // offset k of a row with dx = -1, 0, +1 uses A_{+1}, A_0, A_{-1}
#define C3H_MF3(BF, K0, KS)                                                                              \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                                     \
    const mf_v4i b = ks ? BF.template frag<0, 1>() : BF.template frag<0, 0>();                          \
    acc[K0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2][ks], b, acc[K0], 0, 0, 0);                     \
    acc[K0 + KS] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1][ks], b, acc[K0 + KS], 0, 0, 0);          \
    acc[K0 + 2 * KS] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0][ks], b, acc[K0 + 2 * KS], 0, 0, 0);  \
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1][ks], A[1][ks], acc[13], 0, 0, 0);  // own channels
    // (-1, 0, 0): the unshifted dz = 0 row against A_{+1}
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2][ks], ks ? c0.template frag<0, 1>() : c0.template frag<0, 0>(),
                                                   acc[12], 0, 0, 0);
  }
  MfRow2<-R, 0, 0> rm;  // dz = -1, dy = -1: k = 3 (dx + 1)
  rm.issue(pp + o - pw16);
  cm.pin();
  C3H_MF3(cm, 9, 1)
  MfRow2<0, 0, 0> r0;  // dz = -1, dy = 0: k = 3 (dx + 1) + 1
  r0.issue(pp + o);
  rm.pin();
  C3H_MF3(rm, 0, 3)
  MfRow2<R, 0, 0> rp;  // dz = -1, dy = +1: k = 3 (dx + 1) + 2
  rp.issue(pp + o + pw16);
  r0.pin();
  C3H_MF3(r0, 1, 3)
  rp.pin();
  C3H_MF3(rp, 2, 3)
#undef C3H_MF3
}
template <int R>
__device__ __forceinline__ void mf_layer_ksteps2(const uint8_t* pp, const uint8_t* pc, const mf_u4 (&mk)[2],
                                                 int pw16, int h4, mf_v4i (&acc)[kMfK]) {
  const int o = 32 * h4;
  mf_v4i A0, A1;
#define C3H_MF2(ROW, DX, K)                                                                                 \
  acc[K] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, ROW.template frag<DX, 0>(), acc[K], 0, 0, 0);      \
  acc[K] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, ROW.template frag<DX, 1>(), acc[K], 0, 0, 0);
  if (C3H_MF_PREFETCH) {
    MfRow2<0, -1, 0> c0;   // dz = 0, dy = 0: the centres and dx = -1
    MfRow2<-R, -1, 1> cm;  // dz = 0, dy = -1: k = 9 + dx + 1
    c0.issue(pc + o);
    cm.issue(pc + o - pw16);
    c0.pin();
    const mf_v4i a0 = c0.template frag<0, 0>(), a1 = c0.template frag<0, 1>();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      A0[i] = (int)(((uint32_t)a0[i] & mk[0][i]) | (0x80808080u & ~mk[0][i]));
      A1[i] = (int)(((uint32_t)a1[i] & mk[1][i]) | (0x80808080u & ~mk[1][i]));
    }
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, A0, acc[13], 0, 0, 0);  // own channels
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, A1, acc[13], 0, 0, 0);
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, c0.template frag<-1, 0>(), acc[12], 0, 0, 0);  // (-1, 0, 0)
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, c0.template frag<-1, 1>(), acc[12], 0, 0, 0);
    MfRow2<-R, -1, 1> rm;  // dz = -1, dy = -1: k = 3 (dx + 1)
    rm.issue(pp + o - pw16);
    cm.pin();
    C3H_MF2(cm, -1, 9)
    C3H_MF2(cm, 0, 10)
    C3H_MF2(cm, 1, 11)
    MfRow2<0, -1, 1> r0;  // dz = -1, dy = 0
    r0.issue(pp + o);
    rm.pin();
    C3H_MF2(rm, -1, 0)
    C3H_MF2(rm, 0, 3)
    C3H_MF2(rm, 1, 6)
    MfRow2<R, -1, 1> rp;  // dz = -1, dy = +1
    rp.issue(pp + o + pw16);
    r0.pin();
    C3H_MF2(r0, -1, 1)
    C3H_MF2(r0, 0, 4)
    C3H_MF2(r0, 1, 7)
    rp.pin();
    C3H_MF2(rp, -1, 2)
    C3H_MF2(rp, 0, 5)
    C3H_MF2(rp, 1, 8)
    return;
  }
  {
    // dz = 0: row 0 (the centres and dx = -1)
    MfRow2<0, -1, 0> c0;
    c0.load(pc + o);
    const mf_v4i a0 = c0.template frag<0, 0>(), a1 = c0.template frag<0, 1>();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      A0[i] = (int)(((uint32_t)a0[i] & mk[0][i]) | (0x80808080u & ~mk[0][i]));
      A1[i] = (int)(((uint32_t)a1[i] & mk[1][i]) | (0x80808080u & ~mk[1][i]));
    }
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, A0, acc[13], 0, 0, 0);  // own channels
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, A1, acc[13], 0, 0, 0);
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, c0.template frag<-1, 0>(), acc[12], 0, 0, 0);  // (-1, 0, 0)
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, c0.template frag<-1, 1>(), acc[12], 0, 0, 0);
  }
  {
    MfRow2<-R, -1, 1> cm;  // dz = 0, dy = -1: k = 9 + dx + 1
    cm.load(pc + o - pw16);
    C3H_MF2(cm, -1, 9)
    C3H_MF2(cm, 0, 10)
    C3H_MF2(cm, 1, 11)
  }
  {
    MfRow2<-R, -1, 1> r;  // dz = -1, dy = -1: k = 3 (dx + 1)
    r.load(pp + o - pw16);
    C3H_MF2(r, -1, 0)
    C3H_MF2(r, 0, 3)
    C3H_MF2(r, 1, 6)
  }
  {
    MfRow2<0, -1, 1> r;  // dz = -1, dy = 0
    r.load(pp + o);
    C3H_MF2(r, -1, 1)
    C3H_MF2(r, 0, 4)
    C3H_MF2(r, 1, 7)
  }
  {
    MfRow2<R, -1, 1> r;  // dz = -1, dy = +1
    r.load(pp + o + pw16);
    C3H_MF2(r, -1, 2)
    C3H_MF2(r, 0, 5)
    C3H_MF2(r, 1, 8)
  }
#undef C3H_MF2
}

#ifndef C3H_MF_OCCMASK
#define C3H_MF_OCCMASK 1  // layer conversion: empty voxels restored by a per-dword mask, not a per-read select
#endif
#ifndef C3H_MF_PBASE
#define C3H_MF_PBASE 1  // per-item grid offsets formed once per tile (layer L adds L x the z stride; 2.5 % on config 5)
#endif
#ifndef C3H_MF_SHAPE_CACHE
#define C3H_MF_SHAPE_CACHE 1  // the tile shape's mask and item map kept across same-shape tiles
#endif
#ifndef C3H_MF_LOADX4
#define C3H_MF_LOADX4 1  // a layer item whose 4 words all lie in the grid: one 16-B load
#endif
#ifndef C3H_MF_U32
#define C3H_MF_U32 0  // two-step layers: dx = +-1 and unaligned fragments as byte-offset ds_read_b32
#endif
// Diagnostics: the two-step layers with every fragment not on a 16-byte boundary read as
// four 32-bit LDS loads at its byte offset (each fenced from its neighbours so the compiler
// does not merge them) instead of whole blocks + v_alignbyte: 68 fewer VALU per layer, but
// a ds_read_b32 off a 4-byte boundary is replayed, and config 5 took 11.2 ms instead of
// 1.43 (profiles/r4/config5_ab/): the alignbyte form stays.
typedef uint32_t __attribute__((aligned(1))) mf_u32_ua;
__device__ __forceinline__ uint32_t mf_ld32(const uint8_t* p) {
  const uint32_t v = *reinterpret_cast<const mf_u32_ua*>(p);
  mf_compiler_fence();
  return v;
}
template <int OFF>
__device__ __forceinline__ mf_v4i mf_frag32(const uint8_t* row) {
  if constexpr ((OFF & 15) == 0) {
    const mf_u4 v = *reinterpret_cast<const mf_u4*>(__builtin_assume_aligned(row + OFF, 16));
    return mf_v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
  } else {
    mf_v4i f;
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = (int)mf_ld32(row + OFF + 4 * i);
    return f;
  }
}
// a plane row's fragments dx = -1 .. NDX - 2 of both K steps: 8 NDX loads issued together
// (from row + DYR - 1, so every offset is a non-negative immediate)
template <int DYR, int NDX>
__device__ __forceinline__ void mf_rowu(const uint8_t* row, mf_v4i (&f)[NDX][2]) {
  const uint8_t* b = row + DYR - 1;
#pragma unroll
  for (int d = 0; d < NDX; ++d)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) f[d][ks][i] = (int)mf_ld32(b + d + 16 * ks + 4 * i);
}
template <int R>
__device__ __forceinline__ void mf_layer_ksteps2u(const uint8_t* pp, const uint8_t* pc, const mf_u4 (&mk)[2],
                                                  int pw16, int h4, mf_v4i (&acc)[kMfK]) {
  const int o = 32 * h4;
  const uint8_t* c0 = static_cast<const uint8_t*>(__builtin_assume_aligned(pc + o, 16));
  mf_v4i A0, A1;
  {
    const mf_u4 a0 = *reinterpret_cast<const mf_u4*>(c0), a1 = *reinterpret_cast<const mf_u4*>(c0 + 16);
    mf_v4i fl[1][2];
    mf_rowu<0, 1>(c0, fl);  // dx = -1
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      A0[i] = (int)((a0[i] & mk[0][i]) | (0x80808080u & ~mk[0][i]));
      A1[i] = (int)((a1[i] & mk[1][i]) | (0x80808080u & ~mk[1][i]));
    }
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, A0, acc[13], 0, 0, 0);  // own channels
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, A1, acc[13], 0, 0, 0);
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, fl[0][0], acc[12], 0, 0, 0);  // (-1, 0, 0)
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, fl[0][1], acc[12], 0, 0, 0);
  }
  auto row3 = [&](const mf_v4i (&f)[3][2], int k0, int kstep) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      acc[k0 + kstep * d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, f[d][0], acc[k0 + kstep * d], 0, 0, 0);
      acc[k0 + kstep * d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, f[d][1], acc[k0 + kstep * d], 0, 0, 0);
    }
  };
  {
    mf_v4i f[3][2];
    mf_rowu<-R, 3>(pc + o - pw16, f);  // dz = 0, dy = -1: k = 9 + dx + 1
    row3(f, 9, 1);
  }
  {
    mf_v4i f[3][2];
    mf_rowu<-R, 3>(pp + o - pw16, f);  // dz = -1, dy = -1: k = 3 (dx + 1)
    row3(f, 0, 3);
  }
  {
    mf_v4i f[3][2];
    mf_rowu<0, 3>(pp + o, f);  // dz = -1, dy = 0
    row3(f, 1, 3);
  }
  {
    mf_v4i f[3][2];
    mf_rowu<R, 3>(pp + o + pw16, f);  // dz = -1, dy = +1
    row3(f, 2, 3);
  }
}

#ifndef C3H_MF_TR
#define C3H_MF_TR 1  // two-step layers as a record image read by ds_read_b64_tr_b8 (round 6)
#endif
#ifndef C3H_MF_BFI
#define C3H_MF_BFI 1  // record path: the centre masks as one v_bfi_b32 per dword
#endif
#ifndef C3H_MF_B96
#define C3H_MF_B96 0  // record path: 12-byte record stores, the padding dword written once per tile (slower: 1.09 vs 1.01 ms)
#endif
#ifndef C3H_MF_BUFLD
#define C3H_MF_BUFLD 1  // record path: branch-free raw buffer loads of the layer words
#endif
#ifndef C3H_MF_PLSWAP
#define C3H_MF_PLSWAP 0  // epilogue: row 15's column sums broadcast by two permlane swaps, not ds_bpermute (correct, measured neutral)
#endif
#ifndef C3H_MF_ST16
#define C3H_MF_ST16 1  // fp16 rows: the epilogue stages halves (8-byte LDS stores) instead of floats
#endif
#ifndef C3H_MF_SRC2
#define C3H_MF_SRC2 1  // f16 epilogue: the bin -> stage table read as u16 pairs (one LDS read per pair)
#endif
#ifndef C3H_MF_UNIWID
#define C3H_MF_UNIWID 1  // the wave index through readfirstlane (scalar tile loop)
#endif
// Record image (round 6).  A two-step layer (pitch 12, 12 rows) is held voxel-major: the
// voxel at position p = row * 12 + col has the 16-byte record at byte 16 p of the slot,
// bytes 0..11 = its 12 channel bytes (per colour the setColor table dword {sin, cos, beta,
// 1 - beta} ^ 0x80, as the planes order them; 0x80 each for an empty voxel) and bytes
// 12..15 = {0, 0, 0, 1} (the padding rows / columns).  The conversion is then 3 table
// reads and one ds_write_b128 per voxel, with no byte transpose.  The MFMA operands come
// back channel-major through ds_read_b64_tr_b8: in each 16-lane group, lane 2q + p
// supplies the address of record q's bytes 8p .. 8p + 7 (q = 0..7) and lane i receives
// byte i of the 8 records, i.e. channel i at 8 positions (measured, tools/tr8_probe.hip).
// Two reads give a lane's 16 K bytes.  K map: byte j of lane group h in K step ks is
// position 12 + 64 ks + 32 (j >> 3) + 8 h + (j & 7); A, B and the mask use the same
// bijection, so the integer sums are unchanged.  Groups h and h + 1 (one 32-lane half)
// read 128-byte runs 8 records apart, i.e. disjoint 32-bank halves: conflict-free, and so
// is every neighbour offset (it moves all runs together).  The dx shifts stay on the
// masked centre operand (A_s = centre row read at position + s, masked by the centre mask
// of position + s), so a layer reads 5 neighbour rows + 3 centre shifts = 32 tr reads.
// Records 144..151 of a slot (read by the dy = +1 rows beyond the window's centres) are
// constant padding records.
constexpr int kMfRecPos = 152;
#ifndef C3H_MF_TRFENCE
#define C3H_MF_TRFENCE 1  // record K steps: compiler fences hold each row's reads one row ahead
#endif
#ifndef C3H_MF_KSMAJOR
#define C3H_MF_KSMAJOR 1  // record K steps: K step 0's 14 MFMAs, then step 1's (0: row by row, reads one row ahead)
#endif
#define C3H_MFT_FENCE() \
  do {                  \
    if (C3H_MF_TRFENCE) mf_compiler_fence(); \
  } while (0)
typedef int mf_v2i __attribute__((ext_vector_type(2)));
// (x & m) | (0x80808080 & ~m): one v_bfi_b32 (the compiler split it into two bit ops)
__device__ __forceinline__ int mf_bfi80(uint32_t m, uint32_t x) {
#if C3H_MF_BFI
  uint32_t r;
  __asm__("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(0x80808080u));
  return (int)r;
#else
  return (int)((x & m) | (0x80808080u & ~m));
#endif
}
typedef mf_v2i __attribute__((address_space(3))) * mf_lds_v2i;
template <int OFF>
__device__ __forceinline__ mf_v4i mf_trfrag(const uint8_t* base) {
  const mf_v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((mf_lds_v2i)(base + OFF));
  const mf_v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((mf_lds_v2i)(base + OFF + 16 * 32));
  return mf_v4i{lo.x, lo.y, hi.x, hi.y};
}
// pp / pc: this lane's read base in the dz = -1 / dz = 0 slot, 16 (12 + 8 h + q) + 8 p - 192
// bytes past the slot (the -192 keeps every offset a non-negative immediate: the smallest
// is the dy = -1 row of K step 0); mk[s + 1][ks]: the centre mask of A_s
template <int D, int KS>
__device__ __forceinline__ mf_v4i mf_trrow(const uint8_t* b) {
  return mf_trfrag<16 * (64 * KS + D + 12)>(b);
}
__device__ __forceinline__ void mf_layer_ksteps_tr(const uint8_t* pp, const uint8_t* pc, const uint32_t (&mk)[3][2][4],
                                                   mf_v4i (&acc)[kMfK]) {
  // the reads are issued one row ahead of the MFMAs that use them (compiler fences keep
  // the scheduler from hoisting every read of the layer, which spilled)
  mf_v4i A[3][2], X0[2];
  {
    const mf_v4i xm[2] = {mf_trrow<-1, 0>(pc), mf_trrow<-1, 1>(pc)};
    X0[0] = mf_trrow<0, 0>(pc);
    X0[1] = mf_trrow<0, 1>(pc);
    const mf_v4i xp[2] = {mf_trrow<1, 0>(pc), mf_trrow<1, 1>(pc)};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        A[0][ks][i] = mf_bfi80(mk[0][ks][i], (uint32_t)xm[ks][i]);
        A[1][ks][i] = mf_bfi80(mk[1][ks][i], (uint32_t)X0[ks][i]);
        A[2][ks][i] = mf_bfi80(mk[2][ks][i], (uint32_t)xp[ks][i]);
      }
  }
#if C3H_MF_KSMAJOR
  // every K step's 14 MFMAs before the next step's: 14 MFMAs between two into one accumulator
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const mf_v4i bcm = ks ? mf_trrow<-12, 1>(pc) : mf_trrow<-12, 0>(pc);
    const mf_v4i brm = ks ? mf_trrow<-12, 1>(pp) : mf_trrow<-12, 0>(pp);
    const mf_v4i br0 = ks ? mf_trrow<0, 1>(pp) : mf_trrow<0, 0>(pp);
    const mf_v4i brp = ks ? mf_trrow<12, 1>(pp) : mf_trrow<12, 0>(pp);
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1][ks], A[1][ks], acc[13], 0, 0, 0);
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2][ks], X0[ks], acc[12], 0, 0, 0);
#define C3H_MFK(B, K0, KS)                                                                       \
    acc[K0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2][ks], B, acc[K0], 0, 0, 0);              \
    acc[K0 + KS] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1][ks], B, acc[K0 + KS], 0, 0, 0);   \
    acc[K0 + 2 * KS] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0][ks], B, acc[K0 + 2 * KS], 0, 0, 0);
    C3H_MFK(bcm, 9, 1)
    C3H_MFK(brm, 0, 3)
    C3H_MFK(br0, 1, 3)
    C3H_MFK(brp, 2, 3)
#undef C3H_MFK
  }
  return;
#endif
  mf_v4i b0[2] = {mf_trrow<-12, 0>(pc), mf_trrow<-12, 1>(pc)};  // dz = 0, dy = -1
  C3H_MFT_FENCE();
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1][ks], A[1][ks], acc[13], 0, 0, 0);  // own channels
    acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2][ks], X0[ks], acc[12], 0, 0, 0);    // (-1, 0, 0)
  }
  // offset k of a row with dx = -1, 0, +1 uses A_{+1}, A_0, A_{-1}
#define C3H_MFT3(B, K0, KS)                                                                               \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                                      \
    acc[K0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2][ks], B[ks], acc[K0], 0, 0, 0);                  \
    acc[K0 + KS] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1][ks], B[ks], acc[K0 + KS], 0, 0, 0);       \
    acc[K0 + 2 * KS] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0][ks], B[ks], acc[K0 + 2 * KS], 0, 0, 0); \
  }
  mf_v4i b1[2] = {mf_trrow<-12, 0>(pp), mf_trrow<-12, 1>(pp)};  // dz = -1, dy = -1
  C3H_MFT_FENCE();
  C3H_MFT3(b0, 9, 1)  // dz = 0, dy = -1: k = 9 + dx + 1
  b0[0] = mf_trrow<0, 0>(pp);  // dz = -1, dy = 0
  b0[1] = mf_trrow<0, 1>(pp);
  C3H_MFT_FENCE();
  C3H_MFT3(b1, 0, 3)  // dz = -1, dy = -1: k = 3 (dx + 1)
  b1[0] = mf_trrow<12, 0>(pp);  // dz = -1, dy = +1
  b1[1] = mf_trrow<12, 1>(pp);
  C3H_MFT_FENCE();
  C3H_MFT3(b0, 1, 3)  // dz = -1, dy = 0
  C3H_MFT3(b1, 2, 3)  // dz = -1, dy = +1
#undef C3H_MFT3
}

// lane l gets x of lane 48 + (l & 15) (the accumulator's row 15 to every lane group); every
// lane active
__device__ __forceinline__ uint32_t mf_row3_bcast(uint32_t x) {
#if C3H_MF_PLSWAP
  const auto a = __builtin_amdgcn_permlane32_swap(x, x, false, false);     // [1]: rows 2 3 2 3
  const auto b = __builtin_amdgcn_permlane16_swap(a[1], a[1], false, false);  // [1]: rows 3 3 3 3
  return b[1];
#else
  return (uint32_t)__shfl((int)x, 48 + (int)(threadIdx.x & 15), 64);
#endif
}

// plane p -> (type, reference channel); p >= 12 is padding
__device__ __forceinline__ int mf_type(int p) { return (p >> 1) & 1; }
__device__ __forceinline__ int mf_chan(int p) { return 2 * (p >> 2) + (p & 1); }

// wave wid of nw (all waves of this launch for frame fy); smem = mf_lds_bytes(a.mf_pb);
// LOAD = grid-word items per lane of a layer (1 when every tile's layer fits one pass)
template <int LOAD>
__device__ __forceinline__ void c3hlac_mfma_body(const KArgs& a, int wid_, int nw, int fy_, uint32_t* s_tab,
                                                 uint32_t* dyn) {
  const int64_t fy = fy_;
  // the wave index is wave-uniform: the tile loop's loads and the record path's buffer
  // descriptors stay scalar
  const int wid = C3H_MF_UNIWID ? __builtin_amdgcn_readfirstlane(wid_) : wid_;
  const uint32_t* __restrict__ fgrid = a.grids[fy];
  float* __restrict__ ffeat = a.feat + fy * a.s_feat;
  int32_t* __restrict__ fexist = a.exist + fy * a.s_h;
  unsigned long long* facc = a.acc64 ? a.acc64 + fy * a.s_acc : nullptr;
  const uint32_t* ftf = a.tf + fy * a.s_tf;
  const int32_t* __restrict__ fwork = a.work + fy * a.s_work;
  int32_t* frows = a.rows ? a.rows + fy * a.s_h : nullptr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // a sparse frame (the dot4 tile body takes it): out before any table is built, so the
  // launch on a sparse single frame costs its dispatch only
  if (2 * (int)ftf[2 + (a.epoch & 1)] < a.ntiles) return;
  const int PBM = a.mf_pb;
  // channel-byte tables: T_col[v] = {sin, cos, beta, 1 - beta} ^ 0x80 (setColor LUT, thresholds)
  for (int i = threadIdx.x; i < 768; i += kBlock) {
    const int col = i >> 8, v = i & 255;
    const uint32_t l = a.lut[v];
    const int thr = col == 0 ? a.thr_r : (col == 1 ? a.thr_g : a.thr_b);
    const uint32_t be = v > thr ? 1u : 0u;
    s_tab[i] = ((l & 0xffu) | (l & 0xff00u) | (be << 16) | ((be ^ 1u) << 24)) ^ 0x80808080u;
  }
  if (threadIdx.x == 0) s_tab[768] = 0x80808080u;  // an empty voxel (in the 128-byte gap)
  // s_tab: the kernel's static array (3,200 bytes at LDS address 0, so each table read's
  // address is its byte offset); dyn: the dynamic region right after it (byte 3,200)
  uint8_t* const lds_x = reinterpret_cast<uint8_t*>(dyn) - 128;  // byte 3,072 (the layout's origin)
  uint8_t* cplanes = lds_x + 128;  // zeros | ones | 0xff
  for (int i = threadIdx.x; i < 3 * PBM / 4; i += kBlock)
    reinterpret_cast<uint32_t*>(cplanes)[i] = i < PBM / 4 ? 0u : (i < 2 * PBM / 4 ? 0x01010101u : 0xffffffffu);
  uint8_t* wl = lds_x + mf_const_bytes(PBM) + (size_t)wave * mf_wave_stride(PBM);
  uint16_t* s_src = reinterpret_cast<uint16_t*>(lds_x + mf_const_bytes(PBM) +
                                                (size_t)kMfWaves * mf_wave_stride(PBM));
  const bool staged = !a.atomic && a.variant == 981;
  if (staged) {  // bin -> stage index (c3h bin_of's inverse; every bin written once)
    auto sidx = [](int k, int c, int n) { return k * 144 + ((c >> 2) * 12 + n) * 4 + (c & 3); };
    for (int e = threadIdx.x; e < 14 * 2 * 36; e += kBlock) {
      const int k = e / 72, t = (e / 36) & 1, cc = (e / 6) % 6, nn = e % 6;
      const int c = mf_plane(t, cc), n = mf_plane(t, nn);
      if (k < 13) {
        s_src[495 * t + bin981(k, cc, nn)] = (uint16_t)sidx(k, c, n);
      } else {
        const int b = bin_of(t, 13, nn, cc);
        if (b >= 0) s_src[b] = (uint16_t)sidx(13, c, n);
      }
    }
    for (int e = threadIdx.x; e < 12; e += kBlock) {
      const int t = e / 6, cc = e % 6;
      s_src[495 * t + cc] = (uint16_t)(14 * 144 + mf_plane(t, cc));
    }
  }
  __syncthreads();
  const int nwork = (int)ftf[2 + (a.epoch & 1)];
  if (2 * nwork < a.ntiles) return;  // sparse frame: the dot4 tile body takes it
  const int F = a.variant;
  // this lane holds C_k[c = 4 (lane >> 4) + r][lane & 15]
  const int h4k = lane >> 4, nk = lane & 15;
  const bool realk = nk < kMfCh;

  int shape_prev = -1;  // the tile shape whose mask and item map are current (C3H_MF_SHAPE_CACHE)
  int it_row[LOAD], it_q[LOAD];
  uint32_t it_xs[LOAD];
  for (int wi = wid; wi < nwork; wi += nw) {
    const int tile = fwork[wi];
    const int ix = tile % a.ns0, iy = (tile / a.ns0) % a.ns1, iz = tile / (a.ns0 * a.ns1);
    const int32_t* sx = a.segs + 3 * ix;
    const int32_t* sy = a.segs + 3 * (a.seg_stride + iy);
    const int32_t* sz = a.segs + 3 * (2 * a.seg_stride + iz);
    const int x0 = sx[0], lx = sx[1], y0 = sy[0], ly = sy[1], z0 = sz[0], lz = sz[1];
    const int64_t h = sx[2] + (int64_t)sy[2] * a.sbx + (int64_t)sz[2] * a.sbx * a.sby;
    const int TW = lx + 2, TY = ly + 2, PW = mf_pitch(lx), off0 = mf_off0(PW), nks = mf_nks(lx, ly, PW);
    const int PB = mf_plane_bytes(lx, ly);
    const int ipr = PW >> 2, nitem = TY * ipr;
    const int SS = mf_slot_stride(PB);
    const bool two = C3H_MF_TWO && nks == 2 && (PW & 15) == 12;  // mf_layer_ksteps2's layers
    const int gap = two ? C3H_MF_GAP : 0;  // planes 4..11 shifted (banks, see mf_layer_ksteps2)
    uint8_t* mask = wl + kMfSlots * SS;
    const bool trp = C3H_MF_TR && two;  // record image + transposed reads (mf_layer_ksteps_tr)
    // The tile shape's centre mask and item map (divisions by the pitch: ~300 VALU) are
    // built when the shape differs from this wave's previous tile; S-uniform grids give
    // every interior tile one shape (the mask stays in the wave's LDS region, past the
    // epilogue's staging)
    const int shape = lx | (ly << 8);
    if (!C3H_MF_SHAPE_CACHE || shape != shape_prev) {
      shape_prev = shape;
      if (trp) {
        // record path: per lane group h, 24 mask words (s + 1, ks, i) at mask + 96 h; byte
        // b of word i: position 12 + 64 ks + 32 (j >> 3) + 8 h + (j & 7) + s, j = 4 i + b
        for (int d = lane; d < 96; d += 64) {
          const int gh = d / 24, r = d - 24 * gh, s = r / 8 - 1, ks = (r >> 2) & 1, i = r & 3;
          uint32_t m = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int j = 4 * i + b, p = 12 + 64 * ks + 32 * (j >> 3) + 8 * gh + (j & 7) + s;
            const int row = p / 12, col = p - 12 * row;
            m |= (row >= 1 && row <= ly && col >= 1 && col <= lx ? 0xffu : 0u) << (8 * b);
          }
          reinterpret_cast<uint32_t*>(mask)[d] = m;
        }
      } else
      // centre mask of the K positions PW + 4 j + b: rows 1..ly, columns 1..lx
      // (one word more on each side: the shifted centre rows of mf_layer_ksteps2s read them)
      for (int j = lane - 1; j < 16 * nks + 1; j += 64) {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int p = PW + 4 * j + b, row = p / PW, col = p - row * PW;
          m |= (row >= 1 && row <= ly && col >= 1 && col <= lx ? 0xffu : 0u) << (8 * b);
        }
        *reinterpret_cast<uint32_t*>(mask + off0 + PW + 4 * j) = m;
      }
#pragma unroll
      for (int i = 0; i < LOAD; ++i) {
        const int e = lane + 64 * i, row = e / ipr, q = e - row * ipr;
        it_row[i] = e < nitem ? row : -(1 << 20);
        it_q[i] = q;
        uint32_t xs = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) xs |= (4 * q + j < TW ? 1u : 0u) << j;
        it_xs[i] = xs;
      }
    }
    // layer items (row, dword q) of lane + 64 i: x = x0 - 1 + 4 q + j, valid x bits, the
    // row (-1 when out of the tile or the grid) and the item's byte in a plane
    int it_gy[LOAD], it_x[LOAD], it_dst[LOAD];
    uint32_t it_xm[LOAD];
#pragma unroll
    for (int i = 0; i < LOAD; ++i) {
      const int row = it_row[i], q = it_q[i], gy = y0 - 1 + row;
      it_gy[i] = row >= 0 && (unsigned)gy < (unsigned)a.gy ? gy : -1;
      it_x[i] = x0 - 1 + 4 * q;
      it_dst[i] = row >= 0 ? off0 + row * PW + 4 * q : -1;
      uint32_t xm = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) xm |= ((it_xs[i] >> j) & 1u) && (unsigned)(it_x[i] + j) < (unsigned)a.gx ? 1u << j : 0u;
      it_xm[i] = xm;
    }
    uint32_t wv[2][LOAD][4];
#if C3H_MF_PBASE
    // each item's word at layer 0, once per tile (layer L adds L x the z stride)
    const int64_t zst = (int64_t)a.gy * a.gx;
    int64_t it_base[LOAD];
#pragma unroll
    for (int i = 0; i < LOAD; ++i) it_base[i] = ((int64_t)(z0 - 1) * a.gy + it_gy[i]) * a.gx + it_x[i];
#endif
    auto load_layer = [&](int L, uint32_t (&w)[LOAD][4]) {
#if C3H_MF_EXP & 8
      if (L >= 4) return;  // diagnostics: layers 4.. convert stale words (no loads in the layer loop)
#endif
      const int gz = z0 - 1 + L;
      const bool zin = (unsigned)gz < (unsigned)a.gz;
#pragma unroll
      for (int i = 0; i < LOAD; ++i) {
        const bool rowin = zin && it_gy[i] >= 0;
#if C3H_MF_PBASE
        const uint32_t* src = fgrid + (it_base[i] + L * zst);
#else
        const uint32_t* src = fgrid + (((int64_t)gz * a.gy + it_gy[i]) * a.gx + it_x[i]);
#endif
        if (C3H_MF_LOADX4 && rowin && it_xm[i] == 15u) {  // the item's 4 words in the grid: one load
          typedef uint32_t u4a4 __attribute__((ext_vector_type(4), aligned(4)));
          const u4a4 v = *reinterpret_cast<const u4a4*>(src);
          w[i][0] = v.x; w[i][1] = v.y; w[i][2] = v.z; w[i][3] = v.w;
          continue;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) w[i][j] = rowin && ((it_xm[i] >> j) & 1u) ? src[j] : 0u;
      }
    };
    // 12 channel planes of layer L: per voxel and colour one table read gives the 4 channel
    // bytes, a 4 x 4 byte transpose packs them per channel (4 voxels per dword)
    // PBC: the plane stride as a compile-time constant (two-step tiles: 288 bytes, planes
    // 4..11 16 bytes further), so the 12 plane stores take immediate offsets; 0 = runtime
    auto store_layer_t = [&](int L, const uint32_t (&w)[LOAD][4], auto pbc) {
#if C3H_MF_EXP & 2
      return;
#endif
      constexpr int PBC = decltype(pbc)::value;
      const int PBv = PBC ? PBC : PB, gapv = PBC ? C3H_MF_GAP : gap;
      const int SSv = PBC ? mf_slot_stride(PBC) : SS;
      uint8_t* slot = wl + (L % kMfSlots) * SSv;
#pragma unroll
      for (int i = 0; i < LOAD; ++i) {
        if (it_dst[i] < 0) continue;
        // empty voxels read entry 768 (all channels 0, i.e. 0x80 each)
        uint32_t t[3][4];
#if C3H_MF_OCCMASK
        // every voxel reads its colour bytes' entries (an empty word reads entry 0); the empty
        // voxels' bytes are put back to 0x80 per plane dword by the occupancy mask (byte j =
        // 0xff when voxel j's word has its occupancy byte)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // byte address of each colour's entry in one VALU (the byte select of SDWA)
          uint32_t ar, ag, ab;
          __asm__("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
                  : "=v"(ar) : "v"(w[i][j]));
          __asm__("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                  : "=v"(ag) : "v"(w[i][j]));
          __asm__("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
                  : "=v"(ab) : "v"(w[i][j]));
          const uint8_t* tb = reinterpret_cast<const uint8_t*>(s_tab);
          t[0][j] = *reinterpret_cast<const uint32_t*>(tb + ar);
          t[1][j] = *reinterpret_cast<const uint32_t*>(tb + 1024 + ag);
          t[2][j] = *reinterpret_cast<const uint32_t*>(tb + 2048 + ab);
        }
        const uint32_t occ = __builtin_amdgcn_perm(w[i][1], w[i][0], 0x0c0c0703u) |
                             __builtin_amdgcn_perm(w[i][3], w[i][2], 0x07030c0cu);  // 0x01 / 0x00 bytes
        uint32_t occ8 = occ << 8;
        __asm__("" : "+v"(occ8));  // x 255 as a shift and a subtract, not a v_mul_lo_u32
        const uint32_t om = occ8 - occ;
#else
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int col = 0; col < 3; ++col)
            t[col][j] = s_tab[w[i][j] ? col * 256 + ((w[i][j] >> (16 - 8 * col)) & 0xffu) : 768u];
#endif
        uint8_t* dst = slot + it_dst[i];
#pragma unroll
        for (int col = 0; col < 3; ++col) {
          const uint32_t u0 = __builtin_amdgcn_perm(t[col][1], t[col][0], 0x05010400u);
          const uint32_t u1 = __builtin_amdgcn_perm(t[col][1], t[col][0], 0x07030602u);
          const uint32_t u2 = __builtin_amdgcn_perm(t[col][3], t[col][2], 0x05010400u);
          const uint32_t u3 = __builtin_amdgcn_perm(t[col][3], t[col][2], 0x07030602u);
          uint32_t o[4] = {__builtin_amdgcn_perm(u2, u0, 0x05040100u), __builtin_amdgcn_perm(u2, u0, 0x07060302u),
                           __builtin_amdgcn_perm(u3, u1, 0x05040100u), __builtin_amdgcn_perm(u3, u1, 0x07060302u)};
#if C3H_MF_OCCMASK
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) o[s2] = (o[s2] & om) | (0x80808080u & ~om);
#endif
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) *reinterpret_cast<uint32_t*>(dst + (4 * col + s2) * PBv + (col ? gapv : 0)) = o[s2];
        }
      }
    };
    auto store_layer = [&](int L, const uint32_t (&w)[LOAD][4]) {
      if (two && PB == 288) store_layer_t(L, w, std::integral_constant<int, 288>{});
      else store_layer_t(L, w, std::integral_constant<int, 0>{});
    };
    mf_v4i acc[kMfK];
#pragma unroll
    for (int k = 0; k < kMfK; ++k) acc[k] = mf_v4i{0, 0, 0, 0};
    if (trp) {
      // every record's padding dword {0, 0, 0, 1} and the padding records 144..151 of the
      // three slots (the previous tile's staging overwrote them; the conversion writes only
      // a record's 12 channel bytes)
      mf_compiler_fence();
      if (C3H_MF_B96)
        for (int r = lane; r < kMfSlots * kMfRecPos; r += 64) {
          const int sl = r / kMfRecPos, p = r - sl * kMfRecPos;
          *reinterpret_cast<uint32_t*>(wl + sl * SS + 16 * p + 12) = 0x01000000u;
        }
      if (lane < 3 * (kMfRecPos - 144))
        *reinterpret_cast<mf_u4*>(wl + (lane >> 3) * SS + 16 * (144 + (lane & 7))) =
            mf_u4{0x80808080u, 0x80808080u, 0x80808080u, 0x01000000u};
      // this lane's masks (lanes n >= 12, the padding rows: everything kept)
      uint32_t mk[3][2][4];
      {
        const mf_u4* mrow = reinterpret_cast<const mf_u4*>(mask + 96 * h4k);
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const mf_u4 v = mrow[2 * s + ks];
#pragma unroll
            for (int i = 0; i < 4; ++i) mk[s][ks][i] = realk ? v[i] : 0xffffffffu;
          }
      }
      // this lane's voxels of a layer: positions e = lane + 64 i < 144 (row e / 12, column e % 12)
      // (offsets from the tile's corner word: row * gx + col, -1 outside the tile or the grid)
      int ro[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int e = lane + 64 * i, row = e / 12, col = e - 12 * row;
        const int gy = y0 - 1 + row, gx = x0 - 1 + col;
        const bool v = e < 144 && row < ly + 2 && col < lx + 2 && (unsigned)gy < (unsigned)a.gy && (unsigned)gx < (unsigned)a.gx;
        ro[i] = v ? row * a.gx + col : -1;
      }
      const int64_t zst = (int64_t)a.gy * a.gx;
      const uint32_t* tbase = fgrid + (((int64_t)(z0 - 1) * a.gy + (y0 - 1)) * a.gx + (x0 - 1));
      // branch-free: raw buffer loads off the layer's corner word, an invalid item's offset
      // (-4) and a layer outside the grid (no records) read 0 from the buffer's range check;
      // a valid item's word lies in the grid
      auto load_rec = [&](int L, uint32_t (&w)[3]) {
        const int gz = z0 - 1 + L;
        const bool zin = (unsigned)gz < (unsigned)a.gz;
        // (the base and the record count are wave-uniform; readfirstlane keeps the descriptor
        // in SGPRs, where the compiler would otherwise emit a waterfall loop per load)
        const uint64_t lb = reinterpret_cast<uint64_t>(tbase + L * zst);
        const uint64_t lbu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(lb >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lb);
        const int nrec = __builtin_amdgcn_readfirstlane(zin ? 0x7ffffff0 : 0);
#if C3H_MF_BUFLD
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(lbu), (short)0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < 3; ++i) w[i] = __builtin_amdgcn_raw_buffer_load_b32(r, 4 * ro[i], 0, 0);
#else
        (void)lbu;
        (void)nrec;
        const uint32_t* lp = tbase + L * zst;
#pragma unroll
        for (int i = 0; i < 3; ++i) w[i] = zin && ro[i] >= 0 ? lp[ro[i]] : 0u;
#endif
      };
      auto store_rec = [&](int L, const uint32_t (&w)[3]) {
        uint8_t* slot = wl + (L % kMfSlots) * SS;
        const uint8_t* tb = reinterpret_cast<const uint8_t*>(s_tab);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int e = lane + 64 * i;
          if (i == 2 && e >= 144) continue;
          uint32_t ar, ag, ab;
          __asm__("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
                  : "=v"(ar) : "v"(w[i]));
          __asm__("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                  : "=v"(ag) : "v"(w[i]));
          __asm__("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
                  : "=v"(ab) : "v"(w[i]));
          const uint32_t t0 = *reinterpret_cast<const uint32_t*>(tb + ar);
          const uint32_t t1 = *reinterpret_cast<const uint32_t*>(tb + 1024 + ag);
          const uint32_t t2 = *reinterpret_cast<const uint32_t*>(tb + 2048 + ab);
          const bool occ = (w[i] >> 24) != 0u;
#if C3H_MF_B96
          typedef uint32_t mf_u3 __attribute__((ext_vector_type(3)));
          *reinterpret_cast<mf_u3*>(slot + 16 * e) =
              mf_u3{occ ? t0 : 0x80808080u, occ ? t1 : 0x80808080u, occ ? t2 : 0x80808080u};
#else
          *reinterpret_cast<mf_u4*>(slot + 16 * e) =
              mf_u4{occ ? t0 : 0x80808080u, occ ? t1 : 0x80808080u, occ ? t2 : 0x80808080u, 0x01000000u};
#endif
        }
      };
      uint32_t wr[2][3];
      load_rec(0, wr[0]);
      load_rec(1, wr[1]);
      store_rec(0, wr[0]);
      store_rec(1, wr[1]);
      if (2 <= lz) load_rec(2, wr[0]);
      if (3 <= lz) load_rec(3, wr[1]);
      // lane 2 q + p of group h reads record q's bytes 8 p.. (see mf_layer_ksteps_tr)
      const int tro = 16 * (12 + 8 * h4k + ((lane & 15) >> 1)) + 8 * (lane & 1) - 192;
      for (int z = 0; z < lz; ++z) {
        mf_compiler_fence();
        mf_layer_ksteps_tr(wl + ((z % kMfSlots) * SS + tro), wl + (((z + 1) % kMfSlots) * SS + tro), mk, acc);
        mf_compiler_fence();
        if (z + 2 <= lz) {
          if (z & 1) {
            store_rec(z + 2, wr[1]);
            if (z + 4 <= lz) load_rec(z + 4, wr[1]);
          } else {
            store_rec(z + 2, wr[0]);
            if (z + 4 <= lz) load_rec(z + 4, wr[0]);
          }
        }
      }
    } else {
    load_layer(0, wv[0]);
    load_layer(1, wv[1]);
    store_layer(0, wv[0]);
    store_layer(1, wv[1]);
    if (2 <= lz) load_layer(2, wv[0]);
    if (3 <= lz) load_layer(3, wv[1]);
    // this lane's planes at the K origin: real channels from the layer slots, padding rows /
    // columns from the constant planes (12..14 zeros, 15 ones; their mask keeps everything)
    const int korg = off0 + PW;
    const uint8_t* cpad = cplanes + (nk == 15 ? PBM : 0) + korg;
    const uint8_t* pmask = realk ? mask + korg : cplanes + 2 * PBM + korg;
    const int pw16 = PW & ~15;
    mf_u4 mk2[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};  // two-step layers: the mask, once per tile
    uint32_t mk10[10];  // C3H_MF_ASHIFT: the mask words of bytes 32 h - 4 .. 32 h + 36
    if (nks == 2) {
      mf_compiler_fence();  // the mask plane was written above by this wave
      if (C3H_MF_ASHIFT) {
#pragma unroll
        for (int j = 0; j < 10; ++j) mk10[j] = *reinterpret_cast<const uint32_t*>(pmask + 32 * h4k + 4 * (j - 1));
      } else {
        mk2[0] = *reinterpret_cast<const mf_u4*>(__builtin_assume_aligned(pmask + 32 * h4k, 16));
        mk2[1] = *reinterpret_cast<const mf_u4*>(__builtin_assume_aligned(pmask + 32 * h4k + 16, 16));
      }
    }
    for (int z = 0; z < lz; ++z) {
      mf_compiler_fence();  // same-wave LDS accesses complete in order; keep the compiler's too
      const int pn = nk * PB + (nk >= 4 ? gap : 0) + korg;
      const uint8_t* pp = realk ? wl + ((z % kMfSlots) * SS + pn) : cpad;        // dz = -1
      const uint8_t* pc = realk ? wl + (((z + 1) % kMfSlots) * SS + pn) : cpad;  // dz = 0
#if !(C3H_MF_EXP & 1)
      if (two) {  // S <= 10 tiles: pitch 12
        if (C3H_MF_ASHIFT) mf_layer_ksteps2s<12>(pp, pc, mk10, pw16, h4k, acc);
        else if (C3H_MF_U32) mf_layer_ksteps2u<12>(pp, pc, mk2, pw16, h4k, acc);
        else mf_layer_ksteps2<12>(pp, pc, mk2, pw16, h4k, acc);
      } else {
        switch (PW & 15) {
          case 0: mf_layer_ksteps<0>(pp, pc, pmask, pw16, nks, h4k, acc); break;
          case 4: mf_layer_ksteps<4>(pp, pc, pmask, pw16, nks, h4k, acc); break;
          case 8: mf_layer_ksteps<8>(pp, pc, pmask, pw16, nks, h4k, acc); break;
          default: mf_layer_ksteps<12>(pp, pc, pmask, pw16, nks, h4k, acc); break;
        }
      }
#endif
      mf_compiler_fence();
      // layer z + 2 into the plane slot of layer z - 1 (loaded two layers ago), then the
      // loads of layer z + 4 into its registers
      if (z + 2 <= lz) {
        if (z & 1) {
          store_layer(z + 2, wv[1]);
          if (z + 4 <= lz) load_layer(z + 4, wv[1]);
        } else {
          store_layer(z + 2, wv[0]);
          if (z + 4 <= lz) load_layer(z + 4, wv[0]);
        }
      }
    }
    }  // record path / plane path
    mf_compiler_fence();
    // (the lane's coordinates made opaque per tile, so the bin arithmetic below is not
    // hoisted out of the tile loop and held in registers across it)
    int le = lane;
    __asm__ volatile("" : "+v"(le));
    const int h4 = le >> 4, n = le & 15, tn = mf_type(n), nn = mf_chan(n);
    const bool real = n < kMfCh;
    // epilogue from registers.  pos = C[15][15] (positions), rs[r] = C[4 h4 + r][15] = sum of
    // A'_c (the same for every k), cs_k = C_k[15][n]; value = C + 128 (rs + cs) + 128^2 pos
    const uint32_t pos = (uint32_t)__shfl(acc[13][3], 63, 64);
    uint32_t rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rs[r] = (uint32_t)__shfl(acc[13][r], 16 * h4 + 15, 64);
    const uint32_t k2 = 16384u * pos;
#if C3H_MF_EXP & 4
    {  // diagnostics: no bin epilogue (one word keeps the accumulators live)
      uint32_t x = k2;
#pragma unroll
      for (int k = 0; k < kMfK; ++k) x ^= (uint32_t)(acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3]);
      ffeat[h * F + lane] = (float)x;
      continue;
    }
#endif
    if (staged) {
      // every value once, no per-bin branches: v = C + 128 (rs + cs) + 128^2 pos, times the
      // bin's normalisation (same-type products: type 0 -> kNorm1, type 1 -> 1; the
      // zero-order sums: kNorm0 / 1), as a float4 per lane and k; then the row is gathered
      float* sf = reinterpret_cast<float*>(wl);
      mf_compiler_fence();
      const bool slot = real && h4 < 3;
#if C3H_MF_ST16
      if (a.feat16) {  // fp16 rows: every value rounded once (RNE), as the float stage's gather did
        _Float16* sh = reinterpret_cast<_Float16*>(wl);
        auto put4 = [&](_Float16* dst, float x, float y, float z, float w) {
          const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)x) |
                              ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)y) << 16);
          const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)z) |
                              ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)w) << 16);
          *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
        };
        _Float16* slh = sh + (h4 * 12 + n) * 4;
        uint32_t base[4];
        float nrm[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          base[r] = 128u * rs[r] + k2;
          nrm[r] = mf_type(4 * h4 + r) ? 1.0f : kNorm1;
        }
#pragma unroll
        for (int k = 0; k < kMfK; ++k) {
          const uint32_t cs = 128u * mf_row3_bcast((uint32_t)acc[k][3]);
          if (slot)
            put4(slh + 144 * k, (float)((uint32_t)acc[k][0] + base[0] + cs) * nrm[0],
                 (float)((uint32_t)acc[k][1] + base[1] + cs) * nrm[1], (float)((uint32_t)acc[k][2] + base[2] + cs) * nrm[2],
                 (float)((uint32_t)acc[k][3] + base[3] + cs) * nrm[3]);
        }
        if (n == 15 && h4 < 3)
          put4(sh + 14 * 144 + 4 * h4, (float)(rs[0] + 128u * pos) * (mf_type(4 * h4) ? 1.0f : kNorm0),
               (float)(rs[1] + 128u * pos) * (mf_type(4 * h4 + 1) ? 1.0f : kNorm0),
               (float)(rs[2] + 128u * pos) * (mf_type(4 * h4 + 2) ? 1.0f : kNorm0),
               (float)(rs[3] + 128u * pos) * (mf_type(4 * h4 + 3) ? 1.0f : kNorm0));
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's values are in LDS
        __builtin_amdgcn_wave_barrier();
        const uint16_t* shu = reinterpret_cast<const uint16_t*>(wl);
        uint32_t* out2 = reinterpret_cast<uint32_t*>(a.feat16 + h * a.f16s);
        // (unroll 2: a full unroll with all 8 pairs in flight measured 4 % slower)
#pragma unroll 2
        for (int i = lane; i < (a.f16s >> 1); i += 64) {  // the padding to f16s as zeros
          const uint32_t sp = 2 * i + 1 < 982 ? reinterpret_cast<const uint32_t*>(s_src)[i] : 0u;
          const uint32_t lo = 2 * i < 981 ? (uint32_t)shu[sp & 0xffffu] : 0u;
          const uint32_t hi = 2 * i + 1 < 981 ? (uint32_t)shu[sp >> 16] : 0u;
          out2[i] = lo | (hi << 16);
        }
        if (wid == 0 && lane == 0) *a.feat16_flag = 1u;
        mf_compiler_fence();  // the next tile's layers overwrite the stage after these reads
        goto staged_done;
      }
#endif
      {
      float* sl = sf + (h4 * 12 + n) * 4;
      uint32_t base[4];
      float nrm[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        base[r] = 128u * rs[r] + k2;
        nrm[r] = mf_type(4 * h4 + r) ? 1.0f : kNorm1;
      }
#pragma unroll
      for (int k = 0; k < kMfK; ++k) {
        const uint32_t cs = 128u * (uint32_t)__shfl(acc[k][3], 48 + n, 64);
        if (slot) {
          float4 v;
          v.x = (float)((uint32_t)acc[k][0] + base[0] + cs) * nrm[0];
          v.y = (float)((uint32_t)acc[k][1] + base[1] + cs) * nrm[1];
          v.z = (float)((uint32_t)acc[k][2] + base[2] + cs) * nrm[2];
          v.w = (float)((uint32_t)acc[k][3] + base[3] + cs) * nrm[3];
          *reinterpret_cast<float4*>(sl + 144 * k) = v;
        }
      }
      if (n == 15 && h4 < 3) {  // zero order: the channel sums rs + 128 pos
        float4 v;
        v.x = (float)(rs[0] + 128u * pos) * (mf_type(4 * h4) ? 1.0f : kNorm0);
        v.y = (float)(rs[1] + 128u * pos) * (mf_type(4 * h4 + 1) ? 1.0f : kNorm0);
        v.z = (float)(rs[2] + 128u * pos) * (mf_type(4 * h4 + 2) ? 1.0f : kNorm0);
        v.w = (float)(rs[3] + 128u * pos) * (mf_type(4 * h4 + 3) ? 1.0f : kNorm0);
        *reinterpret_cast<float4*>(sf + 14 * 144 + 4 * h4) = v;
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's values are in LDS
      __builtin_amdgcn_wave_barrier();
      if (a.feat16) {  // fp16 search precision: the row as f16 pairs (half the bytes)
        uint32_t* out2 = reinterpret_cast<uint32_t*>(a.feat16 + h * a.f16s);
#pragma unroll 2
        for (int i = lane; i < (a.f16s >> 1); i += 64) {  // the padding to f16s as zeros
#if C3H_MF_SRC2
          const uint32_t sp = 2 * i + 1 < 982 ? reinterpret_cast<const uint32_t*>(s_src)[i] : 0u;
          const _Float16 lo = 2 * i < 981 ? (_Float16)sf[sp & 0xffffu] : (_Float16)0.0f;
          const _Float16 hi = 2 * i + 1 < 981 ? (_Float16)sf[sp >> 16] : (_Float16)0.0f;
#else
          const _Float16 lo = 2 * i < 981 ? (_Float16)sf[s_src[2 * i]] : (_Float16)0.0f;
          const _Float16 hi = 2 * i + 1 < 981 ? (_Float16)sf[s_src[2 * i + 1]] : (_Float16)0.0f;
#endif
          out2[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
        }
        if (wid == 0 && lane == 0) *a.feat16_flag = 1u;
      } else {
        float* out = ffeat + h * F;
#pragma unroll 4
        for (int i = lane; i < 981; i += 64) out[i] = sf[s_src[i]];
      }
      mf_compiler_fence();  // the next tile's planes overwrite sf after these reads
      }
#if C3H_MF_ST16
    staged_done:;
#endif
    } else if (a.atomic || F == 981) {
      float* out = ffeat + h * F;
      unsigned long long* hacc = a.atomic ? facc + h * 981 : nullptr;
      // 981 rows are staged in the wave's (now idle) plane slots and stored coalesced: a
      // lane's bins are scattered over the row, 56 scattered dword stores per lane were
      // ~0.25 ms of a 512^3 frame
      float* sf = reinterpret_cast<float*>(wl);
      mf_compiler_fence();
      auto emit = [&](int bin, uint32_t v) {
        if (hacc) {
          if (v) atomicAdd(&hacc[bin], (unsigned long long)v);
        } else {
          sf[bin] = (float)v * norm981(bin);
        }
      };
#pragma unroll
      for (int k = 0; k < kMfK; ++k) {
        const uint32_t cs = (uint32_t)__shfl(acc[k][3], 48 + n, 64);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 4 * h4 + r;
          if (c >= kMfCh) continue;
          const int tc = mf_type(c), cc = mf_chan(c);
          const uint32_t v = (uint32_t)acc[k][r] + 128u * (rs[r] + cs) + k2;
          if (k < 13) {
            if (real && tc == tn) emit(495 * tc + bin981(k, cc, nn), v);
          } else if (real) {
            if (tc == 0 && tn == 0) {
              if (cc <= nn) emit(474 + tri6(cc, nn), v);
            } else if (tc == 1 && tn == 1) {
              if (cc <= 1 && nn >= 2) emit(969 + 4 * cc + (nn - 2), v);
              else if ((cc == 2 || cc == 3) && nn >= 4) emit(977 + 2 * (cc - 2) + (nn - 4), v);
            }
          } else if (n == 15) {  // zero order: sum of the channel
            emit(tc ? 495 + cc : cc, rs[r] + 128u * pos);
          }
        }
      }
      if (!hacc) {
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's bins are in LDS
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < 981; i += 64) out[i] = sf[i];
        mf_compiler_fence();  // the next tile's planes overwrite sf after these reads
      }
    } else {  // 117: first-order bins summed over the 13 offsets (color_chlac.hpp:1647-1743)
      float* out = ffeat + h * F;
      uint32_t s1[4] = {0, 0, 0, 0};
      int csum = 0;
#pragma unroll
      for (int k = 0; k < 13; ++k) {
        csum += acc[k][3];
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[r] += (uint32_t)acc[k][r];
      }
      const uint32_t cs1 = (uint32_t)__shfl(csum, 48 + n, 64);
      const uint32_t cs0 = (uint32_t)__shfl(acc[13][3], 48 + n, 64);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 4 * h4 + r;
        if (c >= kMfCh) continue;
        const int tc = mf_type(c), cc = mf_chan(c);
        if (real) {
          if (tc == tn) {
            const int i = (tc ? 69 : 6) + 6 * cc + nn;
            out[i] = (float)(s1[r] + 128u * (13u * rs[r] + cs1) + 13u * k2) * norm117(i);
          }
          const uint32_t v0 = (uint32_t)acc[13][r] + 128u * (rs[r] + cs0) + k2;
          int i = -1;
          if (tc == 0 && tn == 0) {
            if (cc <= nn) i = 42 + tri6(cc, nn);
          } else if (tc == 1 && tn == 1) {
            if (cc <= 1 && nn >= 2) i = 105 + 4 * cc + (nn - 2);
            else if ((cc == 2 || cc == 3) && nn >= 4) i = 113 + 2 * (cc - 2) + (nn - 4);
          }
          if (i >= 0) out[i] = (float)v0 * norm117(i);
        } else if (n == 15) {
          const int i = tc ? 63 + cc : cc;
          out[i] = (float)(rs[r] + 128u * pos) * norm117(i);
        }
      }
    }
    if (!a.atomic && lane == 15)  // exist_voxel_num from the zero-order r sums (search_c3_hlac.h:60-61)
      fexist[h] = exist_from((float)(rs[0] + 128u * pos), (float)(rs[1] + 128u * pos));
    if (frows && lane == 0) frows[wi] = (int32_t)h;
  }
}

}  // namespace c3h

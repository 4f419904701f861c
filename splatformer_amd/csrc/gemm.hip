// fp32 MFMA GEMM with fused gather prologue and bias/affine/act/residual
// epilogue -- the dense work of the PTv3 refiner (qkv/proj/MLP/CPE linears,
// embedding, pooling/unpooling projections, output heads) and, through the
// row-gather prologue, the SubMConv3d CPE as an implicit GEMM over the 27
// neighbour offsets.
//
//   Y[m, n] = act( (sum_k A'[m, k] W[n, k] + bias[n]) * scale[n] + shift[n] ) + R[r(m), n]
//
// A' is A (row-major, lda) or, with a gather index G[M, S], the row
// concatenation of S segments of width Kseg: A'[m, s*Kseg + c] =
// A[G[m*S+s], c] (0 when G < 0).  W is torch's Linear layout [N, K].
//
// gfx950 mapping: v_mfma_f32_32x32x2_f32 (exact f32 FMA chains, 157 TF/s
// peak, no xf32 on CDNA4), 256 threads = 4 waves in a 2x2 grid, each wave a
// (BM/2)x(BN/2) sub-tile of 32x32 MFMA blocks; BK = 32 K-slab staged in LDS
// (row stride 36 floats: conflict-free ds_read_b128), double-buffered with
// register prefetch of the next slab.  Lane half h of every MFMA step s
// consumes k = 16h + s, so each lane reads its 16 k-values with 4 x
// ds_read_b128 per 32-row block.
#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;
constexpr int LDS_STRIDE = BK + 4;
constexpr int THREADS = 256;

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_TANH = 3 };

struct GemmArgs {
  int M, N, K;         // K = S * Kseg when gathering
  const float* A;
  long long lda;
  const int* gidx;     // [M, S] or null
  int S, Kseg;
  const float* W;      // [N, K]
  long long ldw;
  const float* bias;   // [N] or null
  const float* scale;  // [N] or null  (folded BatchNorm)
  const float* shift;  // [N] or null
  int act, act_ncols;  // act applies to columns < act_ncols
  const float* R;      // residual [*, ldr] or null
  long long ldr;
  const int* ridx;     // residual row index [M] or null
  float* Y;
  long long ldy;
  float* Ypre;         // optional copy of the pre-residual value
  long long ldypre;
  // grouped GEMM (blockIdx.z): per-group pointer strides (elements)
  long long gA, gW, gB, gY;
  // sparse implicit GEMM: tile row m -> output row out_rows[m]; seg_mask[m] = bitmask of non-empty
  // gather segments of row m (rows pre-sorted by mask so a tile's OR stays small); the K loop only
  // visits the segments present in the tile's OR.
  const int* out_rows;
  const unsigned* seg_mask;
  int gstride;  // row stride of the gather index (elements; == S unless a column of a wider map is used)
  // offset-major sparse conv ("pair mode"): blockIdx.x walks a flat tile list over up to 27 slices;
  // slice k gathers A rows pair_in[pair_off[k] ..] and atomically adds into rows pair_out[...] with the
  // weight slice W + k * slice_w_stride.
  int pair_mode;
  const int* pair_in;
  const int* pair_out;
  int slice_tile_off[28];
  int slice_pair_off[28];
  int num_slices;
  long long slice_w_stride;
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

template <int BM, int BN, bool VEC>
__global__ void __launch_bounds__(THREADS, 2) gemm_kernel(GemmArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2;   // wave sub-tile
  constexpr int MB = WM / 32, NB = WN / 32; // 32x32 MFMA blocks per wave
  constexpr int A_ITERS = BM * BK / 4 / THREADS;
  constexpr int W_ITERS = BN * BK / 4 / THREADS;
  __shared__ __attribute__((aligned(16))) float sA[2][BM * LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) float sW[2][BN * LDS_STRIDE];

  const int g = blockIdx.z;
  const float* __restrict__ A = p.A + g * p.gA;
  const float* __restrict__ Wt = p.W + g * p.gW;
  const float* __restrict__ bias = p.bias ? p.bias + g * p.gB : nullptr;
  float* __restrict__ Y = p.Y + g * p.gY;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  int M = p.M;
  const int* __restrict__ gidx = p.gidx;
  const int* __restrict__ out_rows = p.out_rows;
  if (p.pair_mode) {
    int sl = 0;
    for (int q = 1; q < p.num_slices; ++q)
      if (p.slice_tile_off[q] <= (int)blockIdx.x) sl = q;
    const int base = p.slice_pair_off[sl];
    M = p.slice_pair_off[sl + 1] - base;
    m0 = ((int)blockIdx.x - p.slice_tile_off[sl]) * BM;
    gidx = p.pair_in + base;
    out_rows = p.pair_out + base;
    Wt = p.W + sl * p.slice_w_stride;
  }
  const int K = p.K;
  int nk = (K + BK - 1) / BK;
  __shared__ unsigned tile_mask_s;
  unsigned tile_mask = 0xffffffffu;
  int cps = 1;  // K chunks per gather segment
  if (p.seg_mask) {
    if (tid == 0) tile_mask_s = 0u;
    __syncthreads();
    unsigned mk = 0u;
    for (int r = tid; r < BM; r += THREADS)
      if (m0 + r < M) mk |= p.seg_mask[m0 + r];
    atomicOr(&tile_mask_s, mk);
    __syncthreads();
    tile_mask = tile_mask_s;
    cps = p.Kseg / BK;
    nk = __popc(tile_mask) * cps;
  }
  // logical K chunk -> physical chunk (skips segments absent from the whole tile)
  auto phys_chunk = [&](int j) -> int {
    if (!p.seg_mask) return j;
    int t = j / cps;
    unsigned mm = tile_mask;
    for (int q = 0; q < t; ++q) mm &= mm - 1u;  // drop the t lowest set bits
    return (__ffs(mm) - 1) * cps + (j - t * cps);
  };

  // this thread's staging coordinates: rows (tid>>3) + 32*i, cols (tid&7)*4
  const int lrow = tid >> 3, lcol = (tid & 7) * 4;

  float4 ra[A_ITERS], rw[W_ITERS];

  auto load_tiles = [&](int kt) {
    const int k0 = phys_chunk(kt) * BK;
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i) {
      const int m = m0 + lrow + 32 * i;
      const int k = k0 + lcol;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M) {
        const float* src = nullptr;
        int kk = k;
        if (gidx) {
          const int s = k / p.Kseg;
          kk = k - s * p.Kseg;
          if (s < p.S) {
            const int r = gidx[(long long)m * p.gstride + s];
            if (r >= 0) src = A + (long long)r * p.lda;
          }
        } else {
          src = A + (long long)m * p.lda;
        }
        if (src) {
          if (VEC) {
            if (k < K) v = *reinterpret_cast<const float4*>(src + kk);
          } else {
            if (k + 0 < K) v.x = src[kk + 0];
            if (k + 1 < K) v.y = src[kk + 1];
            if (k + 2 < K) v.z = src[kk + 2];
            if (k + 3 < K) v.w = src[kk + 3];
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < W_ITERS; ++i) {
      const int n = n0 + lrow + 32 * i;
      const int k = k0 + lcol;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n < p.N) {
        const float* src = Wt + (long long)n * p.ldw;
        if (VEC) {
          if (k < K) v = *reinterpret_cast<const float4*>(src + k);
        } else {
          if (k + 0 < K) v.x = src[k + 0];
          if (k + 1 < K) v.y = src[k + 1];
          if (k + 2 < K) v.z = src[k + 2];
          if (k + 3 < K) v.w = src[k + 3];
        }
      }
      rw[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i)
      *reinterpret_cast<float4*>(&sA[buf][(lrow + 32 * i) * LDS_STRIDE + lcol]) = ra[i];
#pragma unroll
    for (int i = 0; i < W_ITERS; ++i)
      *reinterpret_cast<float4*>(&sW[buf][(lrow + 32 * i) * LDS_STRIDE + lcol]) = rw[i];
  };

  floatx16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int h = lane >> 5, l32 = lane & 31;
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tiles(kt + 1);
    const float* a_base = &sA[cur][(wm * WM + l32) * LDS_STRIDE + h * 16];
    const float* w_base = &sW[cur][(wn * WN + l32) * LDS_STRIDE + h * 16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float4 af[MB], wf[NB];
#pragma unroll
      for (int a = 0; a < MB; ++a) af[a] = *reinterpret_cast<const float4*>(a_base + a * 32 * LDS_STRIDE + 4 * c);
#pragma unroll
      for (int b = 0; b < NB; ++b) wf[b] = *reinterpret_cast<const float4*>(w_base + b * 32 * LDS_STRIDE + 4 * c);
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].x, wf[b].x, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].y, wf[b].y, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].z, wf[b].z, acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a].w, wf[b].w, acc[a][b], 0, 0, 0);
        }
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // epilogue
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int n = n0 + wn * WN + b * 32 + l32;
    if (n >= p.N) continue;
    const float bv = bias ? bias[n] : 0.f;
    const float sc = p.scale ? p.scale[n] : 1.f;
    const float sh = p.shift ? p.shift[n] : 0.f;
    const bool do_act = n < p.act_ncols;
#pragma unroll
    for (int a = 0; a < MB; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mt = m0 + wm * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (mt >= M) continue;
        const int m = out_rows ? out_rows[mt] : mt;
        if (p.pair_mode) {  // partial sum of one neighbour offset: accumulate into the output row
          atomicAdd(&Y[(long long)m * p.ldy + n], acc[a][b][r]);
          continue;
        }
        float v = acc[a][b][r] + bv;
        if (p.scale) v = v * sc + sh;
        if (do_act) {
          if (p.act == ACT_GELU) v = gelu_erf(v);
          else if (p.act == ACT_RELU) v = fmaxf(v, 0.f);
          else if (p.act == ACT_TANH) v = tanhf(v);
        }
        if (p.Ypre) p.Ypre[(long long)m * p.ldypre + n] = v;
        if (p.R) {
          const long long rr = p.ridx ? (long long)p.ridx[m] : (long long)m;
          v += p.R[rr * p.ldr + n];
        }
        Y[(long long)m * p.ldy + n] = v;
      }
    }
  }
}

template <int BM, int BN>
void launch(const GemmArgs& a, int groups, bool vec, hipStream_t st) {
  dim3 grid(a.pair_mode ? a.slice_tile_off[a.num_slices] : sfx::ceil_div(a.M, BM), sfx::ceil_div(a.N, BN), groups);
  if (vec)
    gemm_kernel<BM, BN, true><<<grid, THREADS, 0, st>>>(a);
  else
    gemm_kernel<BM, BN, false><<<grid, THREADS, 0, st>>>(a);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" {

// See include/sfx.h for the contract.
int sfx_linear(int M, int N, int K, const float* A, long long lda, const int* gather_idx, int num_segments,
               const float* W, long long ldw, const float* bias, const float* scale, const float* shift, int act,
               int act_ncols, const float* R, long long ldr, const int* residual_idx, float* Y, long long ldy,
               float* Ypre, long long ldypre, int groups, long long group_stride_A, long long group_stride_W,
               long long group_stride_bias, long long group_stride_Y, const int* out_row_idx,
               const unsigned* segment_mask, void* stream) {
  SFX_REQUIRE(M >= 0 && N > 0 && K > 0, "sfx_linear: bad sizes M=%d N=%d K=%d", M, N, K);
  SFX_REQUIRE(act >= 0 && act <= 3, "sfx_linear: bad activation %d", act);
  SFX_REQUIRE(groups >= 1, "sfx_linear: groups < 1");
  if (M == 0) return SFX_OK;
  SFX_REQUIRE(A && W && Y, "sfx_linear: null buffer");
  const int S = gather_idx ? num_segments : 1;
  SFX_REQUIRE(!gather_idx || (S >= 1 && K % S == 0), "sfx_linear: K must be a multiple of num_segments");
  const int Kseg = K / S;
  SFX_REQUIRE(!gather_idx || Kseg % 4 == 0, "sfx_linear: gathered segment width must be a multiple of 4");
  SFX_REQUIRE(ldw >= K && (gather_idx || lda >= K) && ldy >= N, "sfx_linear: leading dimension too small");
  SFX_REQUIRE(!(scale == nullptr) == !(shift == nullptr), "sfx_linear: scale and shift go together");
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.gidx = gather_idx; a.S = S; a.Kseg = Kseg;
  a.W = W; a.ldw = ldw; a.bias = bias; a.scale = scale; a.shift = shift; a.act = act;
  a.act_ncols = act_ncols < 0 ? N : act_ncols; a.R = R; a.ldr = ldr; a.ridx = residual_idx; a.Y = Y; a.ldy = ldy;
  a.Ypre = Ypre; a.ldypre = ldypre; a.gA = group_stride_A; a.gW = group_stride_W; a.gB = group_stride_bias;
  a.gY = group_stride_Y;
  a.out_rows = out_row_idx;
  a.seg_mask = segment_mask;
  a.gstride = S;
  SFX_REQUIRE(!segment_mask || (gather_idx && Kseg % BK == 0 && S <= 32),
              "sfx_linear: segment_mask needs gather_idx, Kseg %% 32 == 0 and <= 32 segments");
  const bool vec = (K % 4 == 0) && (lda % 4 == 0) && (ldw % 4 == 0) && aligned16(A) && aligned16(W) &&
                   (group_stride_A % 4 == 0) && (group_stride_W % 4 == 0);
  hipStream_t st = sfx::as_stream(stream);
  const long long tiles128 = (long long)sfx::ceil_div(M, 128) * sfx::ceil_div(N, 128) * groups;
  if (N <= 64)
    launch<128, 64>(a, groups, vec, st);
  else if (tiles128 >= 512)
    launch<128, 128>(a, groups, vec, st);
  else
    launch<64, 128>(a, groups, vec, st);
  return sfx::check_launch("sfx_linear");
}

// SubMConv3d, offset-major sparse form.  out = bias + x[nbr[:,13]] W_13^T (dense centre launch, plain
// stores), then one launch over the 26 other offsets' pair lists (pairs from sfx_subm_pairs) whose
// partial products are atomically added.  weight: [Cout, 27, Cin] (spconv [Cout,3,3,3,Cin]).
// pair_off_host: 28 host ints (prefix of pair counts per offset, centre slice empty).
int sfx_subm_conv(int n, int cin, int cout, const float* x, long long ldx, const int* nbr, const float* weight,
                  const float* bias, const int* pair_in, const int* pair_out, const int* pair_off_host, float* out,
                  long long ldo, void* stream) {
  SFX_REQUIRE(n >= 0 && cin > 0 && cout > 0, "sfx_subm_conv: bad sizes");
  if (n == 0) return SFX_OK;
  SFX_REQUIRE(x && nbr && weight && out && pair_off_host, "sfx_subm_conv: null buffer");
  SFX_REQUIRE(ldx >= cin && ldo >= cout, "sfx_subm_conv: leading dimension too small");
  hipStream_t st = sfx::as_stream(stream);
  const bool vec = (cin % 4 == 0) && (ldx % 4 == 0) && aligned16(x) && aligned16(weight);
  // 1) centre offset: dense gathered GEMM with bias, plain stores
  GemmArgs a{};
  a.M = n; a.N = cout; a.K = cin; a.A = x; a.lda = ldx; a.gidx = nbr + 13; a.S = 1; a.Kseg = cin; a.gstride = 27;
  a.W = weight + 13ll * cin; a.ldw = 27ll * cin; a.bias = bias; a.act = 0; a.act_ncols = cout; a.Y = out; a.ldy = ldo;
  const long long tiles128 = (long long)sfx::ceil_div(n, 128) * sfx::ceil_div(cout, 128);
  if (cout <= 64) launch<128, 64>(a, 1, vec, st);
  else if (tiles128 >= 512) launch<128, 128>(a, 1, vec, st);
  else launch<64, 128>(a, 1, vec, st);
  int rc = sfx::check_launch("sfx_subm_conv(centre)");
  if (rc) return rc;
  if (!pair_in || pair_off_host[27] == 0) return SFX_OK;
  // 2) the other 26 offsets as one flat tile list
  GemmArgs b = a;
  b.gidx = nullptr; b.bias = nullptr; b.gstride = 1; b.pair_mode = 1; b.pair_in = pair_in; b.pair_out = pair_out;
  b.W = weight; b.slice_w_stride = cin; b.num_slices = 27;
  const int BMp = (cout <= 64) ? 128 : 64;
  int t = 0;
  for (int k = 0; k < 27; ++k) {
    b.slice_pair_off[k] = pair_off_host[k];
    b.slice_tile_off[k] = t;
    t += (pair_off_host[k + 1] - pair_off_host[k] + BMp - 1) / BMp;
  }
  b.slice_pair_off[27] = pair_off_host[27];
  b.slice_tile_off[27] = t;
  b.M = pair_off_host[27];
  if (cout <= 64) launch<128, 64>(b, 1, vec, st);
  else launch<64, 128>(b, 1, vec, st);
  return sfx::check_launch("sfx_subm_conv(pairs)");
}

}  // extern "C"

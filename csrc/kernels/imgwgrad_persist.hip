// Persistent whole-image weight gradient: dW accumulates in registers across
// the images of a workgroup, one flush per workgroup.
//
//   dW[n][tap*CS + c] += scale * sum_{images, pixels p} dY[p][n] * X[p*stride - pad + tap][c]
//   db[n]            += scale * sum dY[p][n]
//
// GEMM view per image: M = N (dY channels, MT 16-row tiles), columns = (tap, c)
// (KC = T*CS, 16-wide column tiles spread over the 8 waves), reduction k = the
// output pixels.  Both operands are read from LDS with ds_read_b64_tr_b16:
//   A(m = n, k = pixel)        from the dY image   dimg[pixel][NPS]
//   B(k = pixel, col = tap, c) from the source     simg[(y, x)][PS] at pixel + tap
// The earlier per-launch kernel (imgconv.hip) re-staged both images for every
// 16-column slab and flushed partial sums per 4 images; here every image is
// staged once per CU (the next one prefetched into registers while this one's
// MFMAs run) and the whole 64 x 800 dW of MNIST conv2 lives in the 8 waves'
// accumulators (7 column tiles x 4 row tiles per wave).
//
// k order inside a 32-step: MFMA operand element j of lane (g = lane>>4) is
// k = 16*(j>>2) + 4*g + (j&3), so each of the two transposed reads of a
// fragment covers 8 CONSECUTIVE pixels per 32-lane half; with the pixel strides
// of both images an odd multiple of 32 bytes those 8 x 32 B land on 8 distinct
// 32 B bank slots (MI355X_MICROARCH.md §LDS: ds_read_b64_tr_b16 is serviced in
// two 32-lane groups) - conflict-free.  Pixels are enumerated row by row with
// OWP (8/16/32) pixels per row so a 32-step spans whole rows; the dummy pixels
// (x >= OW) carry zero dY.
#include "imgconv.h"

#include <stdexcept>
#include <type_traits>
#include <vector>

namespace dtfe {

namespace {

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for_c(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for_c<B + 1, E>(f);
  }
}

struct WPGeom {
  int LH, LW;       // LDS source extent (pixels), row pitch = LW
  int PS;           // source pixel stride (elements): 16 * odd >= CS
  int NPS;          // dY pixel stride (elements): 16 * odd >= N
  int OWP;          // pixels per enumerated output row (8, 16 or 32)
  int nk;           // 32-pixel k-steps per image
  int img_off;      // dY image offset (elements)
  int slack;        // zero elements after the source image (dummy-pixel reads)
  int schunks;      // 16 B source chunks per image
  int dchunks;      // 16 B dY chunks per image (pooled chunks when pooled)
  int ctiles;       // 16-wide column tiles (KC / 16)
};

__host__ __device__ inline int odd16(int e) {  // round up to 16 * odd elements
  int u = (e + 15) / 16;
  return 16 * (u | 1);
}

// floats per workgroup slab of the register-layout partials (tiles + db, rounded to 16 B)
__host__ __device__ inline int wp_part_len(int MT, int CTW, int N) { return 8 * CTW * MT * 256 + (N + 3) / 4 * 4; }

// KG > 1: the 8 waves form KG k-groups x (8/KG) column groups - wave (kg, cg) runs column tiles
// [cg*CTW, +CTW) over the k-steps s = kg (mod KG), and the k-groups' accumulators are summed through
// LDS before the flush.  Small-KC layers (ResNet-20: 9 or 18 column tiles) otherwise leave most
// waves with dead tiles while one or two carry every MFMA (profiles/r5_resnet20_kernels.txt).
template <int MT, int CTW, int NPFS, int NPFD, bool POOLED, int KG = 1, bool BNX = false>
__global__ __launch_bounds__(512) void imgwgrad_persist_kernel(ImgWgradArgs a, WPGeom G) {
  constexpr int THREADS = 512;
  constexpr int CG = 8 / KG;
  static_assert(KG == 1 || KG == 2 || KG == 4 || KG == 8, "k-groups divide the 8 waves");
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* simg = lds;
  bf16* dimg = lds + G.img_off;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int CS = a.CS, PS = G.PS, NPS = G.NPS, LW = G.LW;
  const int T = a.KH * a.KW, KC = T * CS;

  for (int i = tid; i < (G.LH * LW * PS + G.slack) / 8; i += THREADS)
    reinterpret_cast<u32x4_t*>(simg)[i] = u32x4_t{0u, 0u, 0u, 0u};
  for (int i = tid; i < G.nk * 32 * NPS / 8; i += THREADS)
    reinterpret_cast<u32x4_t*>(dimg)[i] = u32x4_t{0u, 0u, 0u, 0u};

  // ---- per-thread staging destinations (identical for every image)
  int sdst[NPFS], ddst[NPFD];
#pragma unroll
  for (int j = 0; j < NPFS; ++j) {
    const int i = tid + j * THREADS;
    sdst[j] = -1;
    if (i < G.schunks) {
      const int cpp = CS / 8, pix = i / cpp, cc = i - pix * cpp;
      const int sy = pix / a.SW, sx = pix - sy * a.SW, ly = sy + a.pad, lx = sx + a.pad;
      if (ly < G.LH && lx < LW) sdst[j] = (ly * LW + lx) * PS + cc * 8;
    }
  }
#pragma unroll
  for (int j = 0; j < NPFD; ++j) {
    const int i = tid + j * THREADS;
    ddst[j] = -1;
    if (i < G.dchunks) {
      const int cpp = a.N / 8, pix = i / cpp, cc = i - pix * cpp;
      int oy, ox;
      if (POOLED) {
        const int PW = a.OW >> 1, py = pix / PW, px = pix - py * PW;
        oy = 2 * py;
        ox = 2 * px;
      } else {
        oy = pix / a.OW;
        ox = pix - oy * a.OW;
      }
      ddst[j] = (oy * G.OWP + ox) * NPS + cc * 8;
    }
  }
  // BatchNorm + ReLU of the source on staging (a.bns; the conv forward saved the statistics): this
  // thread's source chunks are channels [(tid % (CS/8)) * 8, +8) (512 % (CS/8) == 0)
  constexpr bool bnx = BNX;  // (compile-time instance: the plain kernel is unchanged)
  float bsc[8], bsh[8];
  if constexpr (bnx) bn_src_coeffs(a.bns, a.src, CS, (tid % (CS / 8)) * 8, bsc, bsh);
  u32x4_t sreg[NPFS], dreg[NPFD];
  u32x2_t dam[NPFD];
  auto load_img = [&](long b) {
#pragma unroll
    for (int j = 0; j < NPFS; ++j) {
      const long i = tid + j * THREADS;
      if (i < G.schunks) sreg[j] = *reinterpret_cast<const u32x4_t*>(a.src + b * G.schunks * 8 + i * 8);
    }
#pragma unroll
    for (int j = 0; j < NPFD; ++j) {
      const long i = tid + j * THREADS;
      if (i < G.dchunks) {
        const long off = b * G.dchunks * 8 + i * 8;
        if (POOLED) {
          dreg[j] = *reinterpret_cast<const u32x4_t*>(a.dy_pooled + off);
          dam[j] = *reinterpret_cast<const u32x2_t*>(a.dy_argmax + off);
        } else {
          dreg[j] = *reinterpret_cast<const u32x4_t*>(a.dy + off);
        }
      }
    }
  };
  auto write_img = [&]() {
#pragma unroll
    for (int j = 0; j < NPFS; ++j)
      if (sdst[j] >= 0) {
        if constexpr (bnx) *reinterpret_cast<u32x4_t*>(simg + sdst[j]) = bn_relu_chunk(sreg[j], bsc, bsh);
        else *reinterpret_cast<u32x4_t*>(simg + sdst[j]) = sreg[j];
      }
#pragma unroll
    for (int j = 0; j < NPFD; ++j) {
      if (ddst[j] < 0) continue;
      if (!POOLED) {
        *reinterpret_cast<u32x4_t*>(dimg + ddst[j]) = dreg[j];
      } else {
        u32x4_t v[4];
        unpool4(dreg[j], dam[j], v);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          *reinterpret_cast<u32x4_t*>(dimg + ddst[j] + ((qq >> 1) * G.OWP + (qq & 1)) * NPS) = v[qq];
      }
    }
  };

  // ---- per-lane read offsets.  Lane (g, q, p4) of transposed read h covers local k = 16h + 4g + q.
  const int rows_per_step = 32 / G.OWP;
  int koff[2];  // (oy, ox) of local k at step 0 -> source pixel offset (without tap)
  int doff[2];  // dY row offset
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kl = 16 * h + 4 * g + q, oy = kl / G.OWP, ox = kl - oy * G.OWP;
    koff[h] = (oy * a.stride * LW + ox * a.stride) * PS;
    doff[h] = kl * NPS + 4 * p4;
  }
  const int sstep = rows_per_step * a.stride * LW * PS, dstep = 32 * NPS;
  const int kg = wid / CG, cgi = wid - kg * CG;  // (KG == 1: kg = 0, cgi = wid)
  const int ct0 = cgi * CTW;
  int coff[CTW];  // column tile -> tap offset + channel chunk of this lane
#pragma unroll
  for (int c = 0; c < CTW; ++c) {
    int col = (ct0 + c) * 16 + 4 * p4;
    if (col >= KC) col = 0;  // dead tile: read anything, never flushed
    const int tap = col / CS, ch = col - tap * CS, kh = tap / a.KW, kw = tap - kh * a.KW;
    coff[c] = (kh * LW + kw) * PS + ch;
  }
  const int nct = min(CTW, G.ctiles - ct0);  // live column tiles of this wave (wave-uniform)

  f32x4_t acc[MT][CTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < CTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbacc[MT] = {};

  auto tr2 = [](const bf16* p0, const bf16* p1) {
    const s16x4_t h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p0));
    const s16x4_t h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, p1));
    const s16x8_t v = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  };
  auto load_a = [&](int s, bf16x8_t (&af)[MT]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      af[mt] = tr2(dimg + s * dstep + doff[0] + mt * 16, dimg + s * dstep + doff[1] + mt * 16);
  };
  auto load_b = [&](int s, int c) {
    return tr2(simg + s * sstep + koff[0] + coff[c], simg + s * sstep + koff[1] + coff[c]);
  };

  long b = blockIdx.x;
  if (b < a.B) load_img(b);
  __syncthreads();
  for (; b < a.B; b += gridDim.x) {
    if (!(a.diag & 2) || b == blockIdx.x) write_img();
    __syncthreads();
    if (b + gridDim.x < a.B && !(a.diag & 2)) load_img(b + gridDim.x);
    // Software-pipelined k loop: every wave runs all CTW column tiles (a dead tile - past the
    // weight's columns - reads a valid pixel and is never flushed; on MNIST conv2 only wave 7 has
    // dead tiles and its SIMD partner wave 3 keeps that SIMD at the 14-tile load of the others), so
    // the tile loop is straight-line and its reads can be pinned AHEAD of their MFMAs: column tile
    // c+1's B fragment and step s+1's A fragments are in flight while tile c's MFMAs run.  (The
    // data-dependent `break` at the live-tile count made the scheduler wait on each tile's two
    // transposing reads right before its 4 MFMAs: rocprof ablation, 37.7 of the 57.7 us launch in
    // the MFMA loop at ~56 % MFMA utilisation.)
    const int nk = (a.diag & 4) ? 0 : G.nk;
    if (kg < nk) {
      bf16x8_t a_cur[MT], a_nxt[MT], b_cur = load_b(kg, 0);
      load_a(kg, a_cur);
      for (int s = kg; s < nk; s += KG) {
        const int sn = s + KG < nk ? s + KG : s;  // the last step re-reads its own fragments (unused)
        static_for_c<0, CTW>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          bf16x8_t b_nxt;
          if constexpr (c + 1 < CTW) b_nxt = load_b(s, c + 1);
          else b_nxt = load_b(sn, 0);
          if constexpr (c == 0) load_a(sn, a_nxt);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            acc[mt][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_cur[mt], b_cur, acc[mt][c], 0, 0, 0);
          // reads issued ahead of this tile's MFMAs (c == 0: B of tile 1 + the next step's A)
          __builtin_amdgcn_sched_group_barrier(0x100, c == 0 ? 2 + 2 * MT : 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x8, MT, 0);
          b_cur = b_nxt;
        });
        if (KG == 1 && wid == 0) {  // bias gradient from this step's dY fragments (wave-uniform branch)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const s16x8_t v = __builtin_bit_cast(s16x8_t, a_cur[mt]);
            float sum = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sum += bf2f((bf16)v[e]);
            dbacc[mt] += sum;
          }
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a_cur[mt] = a_nxt[mt];
      }
    }
    __syncthreads();
  }
  // ---- flush.  With a workspace: the accumulators in their REGISTER layout - slab
  // [wave][c][mt][lane] of f32x4, one coalesced 16-B store per lane and tile (the (n, col)
  // scatter happens once, in the reduce kernel) - then db[N] after the 8 * CTW * MT tiles.
  // Without: scaled atomics into dw / db.
  if (a.diag & 1) return;
  if constexpr (KG > 1) {
    // k-group partials -> k-group 0 through LDS (the images are consumed: the loop ended on a
    // barrier), summed in k-group order
    f32x4_t* red = reinterpret_cast<f32x4_t*>(lds);
    if (kg > 0) {
      f32x4_t* mine = red + ((kg - 1) * CG + cgi) * CTW * MT * 64 + lane;
      static_for_c<0, CTW * MT>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        mine[i * 64] = acc[i % MT][i / MT];
      });
    }
    __syncthreads();
    if (kg > 0) return;
    for (int q = 1; q < KG; ++q) {
      const f32x4_t* theirs = red + ((q - 1) * CG + cgi) * CTW * MT * 64 + lane;
      static_for_c<0, CTW * MT>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        acc[i % MT][i / MT] += theirs[i * 64];
      });
    }
  }
  if (a.ws) {
    float* part = a.ws + (long)blockIdx.x * wp_part_len(MT, CTW, a.N);
    f32x4_t* pv = reinterpret_cast<f32x4_t*>(part) + (long)cgi * CTW * MT * 64 + lane;
    // dead tiles (past the weight's columns) are neither stored nor reduced
    static_for_c<0, CTW * MT>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if (i / MT < nct) pv[i * 64] = acc[i % MT][i / MT];
    });
    if (KG == 1 && wid == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v = dbacc[mt];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        const int n = mt * 16 + i16;
        if (lane < 16 && n < a.N) part[8 * CTW * MT * 256 + n] = v;
      }
    }
    return;
  }
  static_for_c<0, CTW * MT>([&](auto ic) {
    constexpr int i = decltype(ic)::value, c = i / MT, mt = i % MT;
    const int col = (ct0 + c) * 16 + i16;
    if (c < nct) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = mt * 16 + g * 4 + j;
        if (n < a.N) atomicAdd(a.dw + (long)n * KC + col, acc[mt][c][j] * a.scale);
      }
    }
  });
  if (KG == 1 && wid == 0 && a.db) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v = dbacc[mt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int n = mt * 16 + i16;
      if (lane < 16 && n < a.N) atomicAdd(a.db + n, v * a.scale);
    }
  }
}

// sum of the register-layout partial slabs over the nblk workgroups in a fixed order (16
// strided subsets, then the subsets in order through LDS: bitwise reproducible, no atomics),
// scattered once into dw[n][col] / db[n]
__device__ __forceinline__ void wp_reduce_body(const float* __restrict__ ws, int nblk, int plen, int MT, int CTW,
                                               int KC, int N, float* dw, float* db, float scale, int blk,
                                               f32x4_t (&red)[16][17]) {
  const int c16 = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int v = blk * 16 + c16;  // f32x4 index within a slab
  const int nv = (plen + 3) / 4;
  const int ntile = 8 * CTW * MT * 64;  // f32x4 of the tile region
  // live entries only: a tile past the weight's KC columns was never stored (small convs such as
  // ResNet-20's 3x3x16 use 9 of the 64 tile slots: the slab traffic shrinks with them)
  const bool live = v < nv && (v >= ntile || ((v >> 6) / MT / CTW * CTW + (v >> 6) / MT % CTW) * 16 < KC);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (live) {
    for (int p0 = pg; p0 < nblk; p0 += 16 * 8) {
      f32x4_t x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p0 + 16 * j;
        x[j] = p < nblk ? *reinterpret_cast<const f32x4_t*>(ws + (long)p * plen + 4 * v) : f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += x[j];
    }
  }
  red[pg][c16] = acc;
  __syncthreads();
  if (pg != 0 || !live) return;
  f32x4_t t = red[0][c16];
#pragma unroll
  for (int q = 1; q < 16; ++q) t += red[q][c16];
  if (v < ntile) {
    const int lane = v & 63, r = v >> 6, mt = r % MT, rc = r / MT, c = rc % CTW, w = rc / CTW;
    const int col = (w * CTW + c) * 16 + (lane & 15), n0 = mt * 16 + (lane >> 4) * 4;
    if (col < KC) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n0 + j < N) dw[(long)(n0 + j) * KC + col] = __builtin_fmaf(scale, t[j], dw[(long)(n0 + j) * KC + col]);
    }
  } else if (db) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = (v - ntile) * 4 + j;
      if (n < N) db[n] = __builtin_fmaf(scale, t[j], db[n]);
    }
  }
}

__global__ __launch_bounds__(256) void wp_reduce_kernel(const float* __restrict__ ws, int nblk, int plen, int MT,
                                                        int CTW, int KC, int N, float* dw, float* db, float scale) {
  __shared__ f32x4_t red[16][17];
  wp_reduce_body(ws, nblk, plen, MT, CTW, KC, N, dw, db, scale, blockIdx.x, red);
}

// Several deferred weight-gradient reduces (each its own workspace) in ONE launch: workgroup
// ranges [first[i], first[i + 1]) reduce item i, exactly as its own wp_reduce_kernel launch would
struct WpReduceItem {
  const float* ws; float* dw; float* db; float scale; int nblk, plen, MT, CTW, KC, N;
};
constexpr int WP_GROUP_MAX = 32;
struct WpReduceGroup {
  WpReduceItem it[WP_GROUP_MAX];
  int first[WP_GROUP_MAX + 1];
  int n;
};
__global__ __launch_bounds__(256) void wp_reduce_group_kernel(WpReduceGroup g) {
  __shared__ f32x4_t red[16][17];
  int i = 0;
  while (i + 1 < g.n && (int)blockIdx.x >= g.first[i + 1]) ++i;
  const WpReduceItem& t = g.it[i];
  wp_reduce_body(t.ws, t.nblk, t.plen, t.MT, t.CTW, t.KC, t.N, t.dw, t.db, t.scale, blockIdx.x - g.first[i], red);
}

thread_local std::vector<WpReduceItem> g_wp_deferred;  // queued by deferred launches, flushed together

}  // namespace

__global__ __launch_bounds__(256) void partials_reduce_kernel(const float* __restrict__ ws, int nblk, int len, int nw,
                                                              float* dw, float* db, float scale) {
  __shared__ f32x4_t red[16][17];
  const int c = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int i = (blockIdx.x * 16 + c) * 4;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (i < len) {
    for (int p0 = pg; p0 < nblk; p0 += 16 * 8) {
      f32x4_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p0 + 16 * j;
        v[j] = p < nblk ? *reinterpret_cast<const f32x4_t*>(ws + (long)p * len + i) : f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j];
    }
  }
  red[pg][c] = acc;
  __syncthreads();
  if (pg == 0 && i < len) {
    f32x4_t t = red[0][c];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += red[q][c];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = i + e;
      if (k < nw) dw[k] = __builtin_fmaf(scale, t[e], dw[k]);
      else if (db) db[k - nw] = __builtin_fmaf(scale, t[e], db[k - nw]);
    }
  }
}

void launch_partials_reduce(const float* ws, int nblk, int len, int nw, float* dw, float* db, float scale,
                            hipStream_t s) {
  hipLaunchKernelGGL(partials_reduce_kernel, dim3((len + 63) / 64), dim3(256), 0, s, ws, nblk, len, nw, dw, db, scale);
}

namespace {

WPGeom wp_geom(const ImgWgradArgs& a) {
  WPGeom G;
  G.LH = (a.OH - 1) * a.stride + a.KH;
  G.LW = (a.OW - 1) * a.stride + a.KW;
  G.PS = odd16(a.CS);
  G.NPS = odd16(a.N);
  G.OWP = a.OW <= 8 ? 8 : (a.OW <= 16 ? 16 : 32);
  const int rows = (a.OH + (32 / G.OWP) - 1) / (32 / G.OWP) * (32 / G.OWP);  // enumerated rows
  G.nk = rows * G.OWP / 32;
  // dummy pixels (x in [OW, OWP), rows >= OH) read up to one enumerated row past the image
  G.slack = ((rows - a.OH + 1) * a.stride * G.LW + G.OWP * a.stride + 8) * G.PS;
  G.img_off = (G.LH * G.LW * G.PS + G.slack + 7) / 8 * 8;
  G.schunks = a.SH * a.SW * a.CS / 8;
  const bool pooled = a.dy == nullptr;
  G.dchunks = (pooled ? (a.OH / 2) * (a.OW / 2) : a.OH * a.OW) * a.N / 8;
  G.ctiles = a.KH * a.KW * a.CS / 16;
  return G;
}

size_t wp_lds(const WPGeom& G) { return ((size_t)G.img_off + (size_t)G.nk * 32 * G.NPS) * sizeof(bf16); }

template <int MT, int CTW, bool POOLED, int KG = 1, bool BNX = false>
bool wp_launch(const ImgWgradArgs& a, const WPGeom& G, hipStream_t s) {
  size_t lds = wp_lds(G);
  if (lds > 150 * 1024) return false;
  if ((G.ctiles + CTW - 1) / CTW > 8 / KG) return false;
  if (KG > 1 && a.db) return false;  // (the bias gradient is summed by the k-group-0 waves only)
  const size_t red = (size_t)(KG - 1) * (8 / KG) * CTW * MT * 64 * sizeof(f32x4_t);
  if (red > lds) lds = red;
  if (lds > 160 * 1024) return false;
  const int npfs = (G.schunks + 511) / 512, npfd = (G.dchunks + 511) / 512;
  // at least ~256 output pixels per workgroup: on small maps the per-workgroup partial slab (up to
  // 229 KB, written and re-read by wp_reduce) outweighs one image's work - ResNet-20 stage 3
  // (8x8, B=256): 64 workgroups 18.8 us vs 256: 26.3 (profiles/r5_resnet20_kernels.txt)
  // (k-group configs: ~512 pixels - their per-image MFMA time is shorter; stage 2: 128 workgroups
  // 14.2 us vs 256: 16.0)
  const int px = KG > 1 ? 512 : 256;
  const int ipw = (px + a.OH * a.OW - 1) / (a.OH * a.OW);
  int gcap = a.max_blocks > 0 && a.max_blocks < 256 ? a.max_blocks : 256;
  if ((a.B + ipw - 1) / ipw < gcap) gcap = (a.B + ipw - 1) / ipw;
  const int grid = a.B < gcap ? a.B : gcap;
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    static const int diag = diag_bits("iw");
    ImgWgradArgs ad = a;
    ad.diag = diag;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, s, ad, G);
    if (a.ws) {
      const int plen = wp_part_len(MT, CTW, a.N), KC = a.KH * a.KW * a.CS;
      if (a.defer_reduce) {
        if (g_wp_deferred.size() >= (size_t)WP_GROUP_MAX) throw std::runtime_error("imgwgrad: too many deferred reduces");
        g_wp_deferred.push_back(WpReduceItem{a.ws, a.dw, a.db, a.scale, grid, plen, MT, CTW, KC, a.N});
      } else {
        hipLaunchKernelGGL(wp_reduce_kernel, dim3((plen / 4 + 15) / 16), dim3(256), 0, s, a.ws, grid, plen, MT, CTW,
                           KC, a.N, a.dw, a.db, a.scale);
      }
    }
    return true;
  };
  // prefetch chunks per thread (source, dY): 1, 2 or 4 each
  auto q = [](int n) { return n <= 1 ? 1 : (n <= 2 ? 2 : (n <= 4 ? 4 : 0)); };
  switch (q(npfs) * 8 + q(npfd)) {
    case 9: return go(imgwgrad_persist_kernel<MT, CTW, 1, 1, POOLED, KG, BNX>);
    case 10: return go(imgwgrad_persist_kernel<MT, CTW, 1, 2, POOLED, KG, BNX>);
    case 12: return go(imgwgrad_persist_kernel<MT, CTW, 1, 4, POOLED, KG, BNX>);
    case 17: return go(imgwgrad_persist_kernel<MT, CTW, 2, 1, POOLED, KG, BNX>);
    case 18: return go(imgwgrad_persist_kernel<MT, CTW, 2, 2, POOLED, KG, BNX>);
    case 20: return go(imgwgrad_persist_kernel<MT, CTW, 2, 4, POOLED, KG, BNX>);
    case 33: return go(imgwgrad_persist_kernel<MT, CTW, 4, 1, POOLED, KG, BNX>);
    case 34: return go(imgwgrad_persist_kernel<MT, CTW, 4, 2, POOLED, KG, BNX>);
    case 36: return go(imgwgrad_persist_kernel<MT, CTW, 4, 4, POOLED, KG, BNX>);
    default: return false;
  }
}

}  // namespace

int flush_wgrad_reduces(hipStream_t s) {
  const int n = (int)g_wp_deferred.size();
  if (n == 0) return 0;
  WpReduceGroup g{};
  g.n = n;
  g.first[0] = 0;
  for (int i = 0; i < n; ++i) {
    g.it[i] = g_wp_deferred[i];
    g.first[i + 1] = g.first[i] + (g.it[i].plen / 4 + 15) / 16;
  }
  g_wp_deferred.clear();
  hipLaunchKernelGGL(wp_reduce_group_kernel, dim3(g.first[n]), dim3(256), 0, s, g);
  return n;
}

int pending_wgrad_reduces() { return (int)g_wp_deferred.size(); }

int discard_wgrad_reduces() {
  const int n = (int)g_wp_deferred.size();
  g_wp_deferred.clear();
  return n;
}

long imgwgrad_ws_floats(int N, int KC) {
  const int MT = N > 32 ? 4 : 2, CTW = N > 32 ? 7 : 9;  // the largest wp_launch slabs below
  const long plain = (long)N * KC + N;                   // imgconv1_copies / per-image kernels
  const long reg = wp_part_len(MT, CTW, N);
  return 256L * (plain > reg ? plain : reg);
}

bool launch_imgwgrad_persistent(const ImgWgradArgs& a, hipStream_t s) {
  if (a.CS % 16 || a.N % 8 || a.N > 64 || a.OW > 32 || a.B < 128) return false;
  const bool pooled = a.dy == nullptr;
  if (pooled && ((a.OH | a.OW) & 1)) return false;
  const WPGeom G = wp_geom(a);
  // 8 waves share the column tiles; MNIST conv2: 50 tiles -> 7 per wave.  Few column tiles (<= 9
  // per column group, no bias gradient): k-groups of waves instead (KG, see the kernel)
  const int ctw = (G.ctiles + 7) / 8;
  const bool ks = !a.db && !(diag_bits("iwk") & 1);
  // (BN + ReLU of the source on staging: compile-time instances of the ResNet configurations only)
  const bool bn = a.bns.stats != nullptr;
  if (ks && G.ctiles <= 9 && a.N <= 16 && !pooled)
    return bn ? wp_launch<1, 9, false, 8, true>(a, G, s) : wp_launch<1, 9, false, 8>(a, G, s);
  if (ks && G.ctiles <= 9 && a.N <= 32 && !pooled)
    return bn ? wp_launch<2, 9, false, 8, true>(a, G, s) : wp_launch<2, 9, false, 8>(a, G, s);
  if (ks && G.ctiles <= 18 && a.N <= 32 && !pooled)
    return bn ? wp_launch<2, 9, false, 4, true>(a, G, s) : wp_launch<2, 9, false, 4>(a, G, s);
  if (a.N > 32 && ks && G.ctiles <= 40 && !pooled)
    return bn ? wp_launch<4, 5, false, 1, true>(a, G, s) : wp_launch<4, 5, false>(a, G, s);
  if (bn) return false;
  if (a.N > 32) {
    if (ctw <= 7) return pooled ? wp_launch<4, 7, true>(a, G, s) : wp_launch<4, 7, false>(a, G, s);
    return false;
  }
  if (ctw <= 8) return pooled ? wp_launch<2, 8, true>(a, G, s) : wp_launch<2, 8, false>(a, G, s);
  return false;
}

}  // namespace dtfe

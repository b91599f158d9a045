// Fused gfx950 kernels for the MNIST-CNN training step (fp32 in / fp32 accumulate, exact).
//
// One step = 5 launches at world size 1, 6 when gradient collectives run:
//   F2  on-device batch + conv1+ReLU + conv2+bias+ReLU+maxpool (MFMA)
//   F3  fc1 forward, split-K (MFMA), partials added as int64 fixed point (order-independent)
//   F5  head (fc1 bias+ReLU, fc2, log_softmax+NLL, dlogits, fc2/fc1-bias grads, dh) recomputed in
//       every block + fc1 dgrad/wgrad (MFMA) + ReLU/maxpool-masked dp          -> bucket 0 ready
//       (world size 1: no fc1 weight gradient here -- F5 publishes dh, see F67)
//   F67 conv2 wgrad (F6W blocks, MFMA) and conv2 dgrad + conv1 ReLU mask + conv1 wgrad (F7W
//       blocks) in ONE launch (co-scheduled peer exchange blocks first when that strategy runs);
//       world size 1: its last 192 blocks compute fc1's weight gradient and apply its SGD update
//       (MnistFused::fc1_defer), resident beside the conv blocks at three blocks per CU, so that
//       work left F5's critical path (default; F5 folds it in when the batch exceeds 64)
//   F8  finalize conv grads, reset accumulators                                -> bucket 1 ready
//       (world size > 1 only: at world size 1 its duties are folded into the SGD launch)
//   SGD flat SGD + repack conv2 weights into the MFMA fragment orders of F2 / F7
// (mnist_conv_bwd.hip holds F67 and F8; mnist_engine.cpp sequences them.)
//
// MFMA = v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15]; the C/D tile
// has col = l&15, row = 4*(l>>4) + reg.  Where operands are read as float4 along K the K order
// inside a 16-wide group is permuted (k = 16*s' + 4*g + j for k-step (s', j), lane group
// g = l>>4) identically for A and B -- legal because K is a pure reduction.
//
// Every cross-step duty (weight packing, zeroing accumulators) is folded into a kernel that
// already exists (SGD, F8); the step has no helper launches.  Every cross-block sum is either a
// fixed-order reduction or an int64 fixed-point atomic (mnist_common.h), so a step is bitwise
// reproducible run to run.
//
// Replaces (reference): cuDNN conv/ReLU/pool + cuBLAS linear + log_softmax/NLL + per-tensor
// SGD kernels reached through the PyTorch training loop of
// pytorch/distributed_data_parallel.py:118-152 (north-star MNIST CNN variant).
#include "mnist_common.h"
#include "rng.h"

namespace mx {
namespace mnist {
namespace {

// F7W B operand for (co, ci) = pair i of 2048: U = G w' G^T, w'[a][b] = w[co][ci][2-a][2-b] (the
// data gradient is the full correlation of dY2 with the flipped filter), G = [1 0 0; .5 .5 .5;
// .5 -.5 .5; 0 0 1].  Stored at ((s*2 + half)*64 + lane)*16 + xi for k-step s = co/4,
// lane = (ci & 15) + 16*(co & 3), half = ci/16, xi = 4i + j: one lane's 16 values are contiguous.
__device__ __forceinline__ void wino_dgrad_filter(const MnistFused& f, const Scratch& sc, int i) {
  const int co = i >> 5, ci = i & 31;
  const float* w = f.p + L::w2 + i * 9;  // (co*32 + ci)*9
  float gp[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) gp[a][b] = w[(2 - a) * 3 + (2 - b)];
  float t[4][3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    t[0][b] = gp[0][b];
    t[1][b] = 0.5f * (gp[0][b] + gp[1][b] + gp[2][b]);
    t[2][b] = 0.5f * (gp[0][b] - gp[1][b] + gp[2][b]);
    t[3][b] = gp[2][b];
  }
  float u[16];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    u[4 * a + 0] = t[a][0];
    u[4 * a + 1] = 0.5f * (t[a][0] + t[a][1] + t[a][2]);
    u[4 * a + 2] = 0.5f * (t[a][0] - t[a][1] + t[a][2]);
    u[4 * a + 3] = t[a][2];
  }
  const int lane = (ci & 15) + 16 * (co & 3);
  float4* dst = reinterpret_cast<float4*>(sc.wu + ((((co >> 2) * 2 + (ci >> 4)) * 64 + lane) * 16));
#pragma unroll
  for (int k = 0; k < 4; ++k) dst[k] = make_float4(u[4 * k], u[4 * k + 1], u[4 * k + 2], u[4 * k + 3]);
}

// F2W B operand: U = G w G^T for (co, ci) (forward = plain correlation, no flip), u[4a + b] with
// a the ky-side and b the kx-side Winograd point.  Stored at ((((co/16)*16 + xi)*2 + s/4)*64 +
// lane)*4 + (s&3) for k-step s = ci/4, lane = (co & 15) + 16*(ci & 3): a wave (= 16 output
// channels) reads one float4 per lane per (xi, 4 k-steps).
__device__ __forceinline__ int wv_index(int co, int ci, int xi) {
  const int s = ci >> 2, l = (co & 15) + 16 * (ci & 3);
  return ((((co >> 4) * 16 + xi) * 2 + (s >> 2)) * 64 + l) * 4 + (s & 3);
}
// The F2W Winograd filter of conv2 weight pair (co, ci) (taps w[0..8] = w[co][ci][ky][kx]).
__device__ __forceinline__ void conv2_pack_pair(const Scratch& sc, int pair, const float w[9]) {
  const int co = pair >> 5, ci = pair & 31;
  float t[4][3];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    t[0][b] = w[b];
    t[1][b] = 0.5f * (w[b] + w[3 + b] + w[6 + b]);
    t[2][b] = 0.5f * (w[b] - w[3 + b] + w[6 + b]);
    t[3][b] = w[6 + b];
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    sc.wv[wv_index(co, ci, 4 * a + 0)] = t[a][0];
    sc.wv[wv_index(co, ci, 4 * a + 1)] = 0.5f * (t[a][0] + t[a][1] + t[a][2]);
    sc.wv[wv_index(co, ci, 4 * a + 2)] = 0.5f * (t[a][0] - t[a][1] + t[a][2]);
    sc.wv[wv_index(co, ci, 4 * a + 3)] = t[a][2];
  }
}

// ------------------------------------------------------------------------------------------
// K0 (once, and after any external weight load): pack conv2 weights, zero accumulators.
__global__ __launch_bounds__(256) void k_init(MnistFused f, Scratch sc) {
  const int gtid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  for (int i = gtid; i < 2048; i += gsz) {
    float w[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) w[r] = f.p[L::w2 + i * 9 + r];
    conv2_pack_pair(sc, i, w);
  }
  for (int i = gtid; i < f.B * 128; i += gsz) f.h[i] = 0;
  for (int i = gtid; i < kG1Slabs * 320; i += gsz) sc.g1[i] = 0;
  if (gtid < 64) sc.db2[gtid] = 0;
  if (gtid == 0) *sc.bad = 0;
}

// F2 a1 tile pitches (row 38, channel 141): picked by an exhaustive bank model (32-lane groups,
// bank = dword mod 32) over the two access patterns that dominate F2W's LDS time -- the conv1
// MFMA stores (16 channels x 2 position groups per 32 lanes) and the stage-2 input-transform
// reads (3 channels x 12 tiles): 1,472 -> 576 LDS cycles per block (40 / 176 had 8-way store
// conflicts).
constexpr int kF2RowP = 38, kF2ChP = 141;

// F2W stage 2 (see f2_fwd_kernel): a1 tile [32 ci][4 rows][26] (pitches kF2ChP / kF2RowP) in
// `tile` -> pooled conv2 outputs of pooled row py of image b.
__device__ __forceinline__ void f2_stage2_wino(const MnistFused& f, const Scratch& sc, float* tile, int b, int py,
                                               int w, int lane) {
  const int tid = threadIdx.x;
  // B fragments of points 0, 1: requested here, in flight during the input transform (issued at
  // kernel start they stayed live through stage 1 and the register shuffles around them waited
  // for the loads: vmcnt(0) in the middle of the transform)
  const float4* up = reinterpret_cast<const float4*>(sc.wv) + (size_t)w * 16 * 2 * 64 + lane;
  float4 bc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bc[q] = up[(q >> 1) * 128 + 64 * (q & 1)];
  // (a) input transform: items (ci, t) = it / 12, it % 12, two per thread (384 items)
  float v[2][16];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int it = tid + 256 * k;
    if (it < 384) {
      const int ci = it / 12, t = it - 12 * (it / 12);
      const float* d = tile + ci * kF2ChP + 2 * t;
      float x[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) x[i][j] = d[i * kF2RowP + j];
      float r[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        r[0][j] = x[0][j] - x[2][j];
        r[1][j] = x[1][j] + x[2][j];
        r[2][j] = x[2][j] - x[1][j];
        r[3][j] = x[1][j] - x[3][j];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        v[k][4 * a + 0] = r[a][0] - r[a][2];
        v[k][4 * a + 1] = r[a][1] + r[a][2];
        v[k][4 * a + 2] = r[a][2] - r[a][1];
        v[k][4 * a + 3] = r[a][1] - r[a][3];
      }
    }
  }
  lds_barrier();  // every a1 read done: V overwrites the tile
  // V as [16 xi][32 ci][12 tiles]: item it = 12 ci + t stores to it itself (consecutive lanes,
  // conflict-free; the former [ci][16] pitch put ci and ci + 4 on one bank range, 2-way).  The
  // MFMA's A rows 12..15 (no tile) read the next channel's values: finite, and only rows 0..11
  // of the result are used.
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int it = tid + 256 * k;
    if (it < 384) {
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) tile[xi * 384 + it] = v[k][xi];
    }
  }
  lds_barrier();
  MX_TRACE(f, 0, 3);
  // (b) 16 GEMMs; lane: A row = tile m, k = ci 4s + g; B col = co 16w + m
  const int m = lane & 15, g = lane >> 4;
  // Points are processed in pairs: two independent accumulator chains interleave, so a
  // dependent MFMA never waits on its predecessor's latency; the next pair's B fragments are
  // in flight during the current pair's MFMAs.
  f32x4 acc[16];
#pragma unroll
  for (int xp = 0; xp < 8; ++xp) {
    float4 bn[4] = {bc[0], bc[1], bc[2], bc[3]};
    if (xp < 7) {
#pragma unroll
      for (int q = 0; q < 4; ++q) bn[q] = up[(2 * xp + 2 + (q >> 1)) * 128 + 64 * (q & 1)];
    }
    // keep the next pair's loads here: the scheduler otherwise sinks them into this pair's MFMAs
    // and waits for L2 (vmcnt) inside the pair
    __builtin_amdgcn_sched_barrier(0);
    acc[2 * xp] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[2 * xp + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* a = tile + 2 * xp * 384 + g * 12 + m;  // A[tile m][ci 4s + g]
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      acc[2 * xp] = mfma4(a[48 * s], sel4(bc[s >> 2], s & 3), acc[2 * xp]);
      acc[2 * xp + 1] = mfma4(a[384 + 48 * s], sel4(bc[2 + (s >> 2)], s & 3), acc[2 * xp + 1]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) bc[q] = bn[q];
  }
  MX_TRACE(f, 0, 4);
  // (c) lane holds points xi of tiles 4g + j (j < 4), channel co: inverse transform + pool
  if (g < 3) {
    const int co = 16 * w + m;
    const float bias = f.p[L::b2 + co];
    uint8_t* idx = reinterpret_cast<uint8_t*>(f.idx);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float r0[4], r1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        r0[c] = acc[c][j] + acc[4 + c][j] + acc[8 + c][j];
        r1[c] = acc[4 + c][j] - acc[8 + c][j] - acc[12 + c][j];
      }
      const float y[4] = {r0[0] + r0[1] + r0[2], r0[1] - r0[2] - r0[3], r1[0] + r1[1] + r1[2],
                          r1[1] - r1[2] - r1[3]};  // (dy, dx) = (0,0) (0,1) (1,0) (1,1)
      float best = y[0];
      int q = 0;
#pragma unroll
      for (int e = 1; e < 4; ++e)
        if (y[e] > best) { best = y[e]; q = e; }
      const float vv = best + bias;
      const int o = ((b * 64 + co) * 12 + py) * 12 + 4 * g + j;
      st1(f.pool + o, vv > 0.f ? vv : 0.f, f.wt & 2);
      idx[o] = vv > 0.f ? (uint8_t)q : (uint8_t)4;
    }
  }
}

// ------------------------------------------------------------------------------------------
// F2: [synthetic batch] + conv1 + ReLU + conv2 (32->64, 3x3) + bias + ReLU + maxpool 2x2.
// Block = (image b, pooled row py).  Stage 1 builds the 6 input rows it needs (generated by
// the Philox stream of ops_data.hip synth_batch, or read from x) and recomputes the 4 conv1
// rows feeding this pooled row straight into the LDS tile (a1 rows shared by neighbouring
// blocks are recomputed, 25 MFLOP total); the rows this block owns are published to a1 for the
// weight gradient (F6W), and x for the data gradient's conv1 mask.  The tile [32 ci][4 rows][26]
// has row pitch kF2RowP and channel pitch kF2ChP (see their definition).
//
// Stage 2 is conv2 as Winograd F(2x2,3x3).  The
// block's 12 pooling windows are exactly 12 Winograd output tiles, so the per-tile inverse
// transform ends in the 2x2 max-pool.  V = B^T d B of every (tile, ci) goes to LDS over the a1
// tile ([16 xi][32 ci][12 tiles]; the MFMA's A rows 12..15 are unused), then 16 GEMMs (one per Winograd
// point) M = 16 tiles x N = 64 co (wave w: 16 co) x K = 32 ci: 128 MFMAs per wave instead of
// 216.  The 16 accumulators of a lane hold all 16 points of its (tile, co), so A^T M A, bias,
// max-pool, argmax and ReLU happen in registers.
__global__ __launch_bounds__(256) void f2_fwd_kernel(MnistFused f, Scratch sc) {
  MX_TRACE(f, 0, 0);
  __shared__ float tile[16 * 32 * 16];
  __shared__ float xs[6 * 28];
  __shared__ float w1s[288 + 32];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // an image's 12 blocks share one XCD L2
  const int b = bid / 12, py = bid - b * 12;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row0 = 2 * py;  // first input row of this block's conv1 rows
  // ---- stage 1a: input rows row0 .. row0+5 (+ publish the rows this block owns).  Every global
  // operand of stage 1 is requested in ONE round trip: the batch counter, conv1's weights and --
  // synthetic data -- the 6 template rows of ALL 10 classes (the label, a function of the counter,
  // then selects one in registers), instead of counter -> label -> template -> weights as four
  // dependent trips.  Loads use clamped lanes (no per-lane branches) and the B fragments of stage 2 are
  // issued after them, so waiting for stage 1 never drains the fragments (vmcnt counts in order).
  const int own_lo = row0, own_hi = py == 11 ? 28 : row0 + 2;  // x rows written by this block
  const int t42 = min(tid, 41), d = row0 * 28 + t42 * 4;
  float w1v[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) w1v[k] = f.p[L::w1 + min(tid + 256 * k, 319)];
  // (both data sources are requested whatever f.synth says -- counter, templates and x always
  // exist -- so no load sits behind a branch whose join would make the waitcnt pass drain the
  // B fragments too)
  const uint32_t ctr = (uint32_t)*f.counter;
  float4 tv[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) tv[c] = *reinterpret_cast<const float4*>(f.tmpl + c * 784 + d);
  const float4 xv = *reinterpret_cast<const float4*>(f.x + b * 784 + d);
  __builtin_amdgcn_sched_barrier(0);  // every stage-1 load issued before the counter is consumed
  {  // branch-free in f.synth (a branch would let the compiler sink the template loads behind
     // the counter's round trip): both sources are formed, one is kept
    const uint2 key = synth_key(f.seed);
    const int label = synth_label(ctr, b, 10, key);
    // masked sum, not `label == c ? tv[c] : t` (hipcc turns that select chain into tv[label]:
    // a dynamically indexed array in scratch memory)
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < 10; ++c) {
      const float mk = (float)(label == c);
      t.x = fmaf(mk, tv[c].x, t.x);
      t.y = fmaf(mk, tv[c].y, t.y);
      t.z = fmaf(mk, tv[c].z, t.z);
      t.w = fmaf(mk, tv[c].w, t.w);
    }
    const uint4 r = synth_noise4(ctr, b, d, key);
    const float4 sv = make_float4(0.5f * t.x + 0.5f * u01(r.x), 0.5f * t.y + 0.5f * u01(r.y),
                                  0.5f * t.z + 0.5f * u01(r.z), 0.5f * t.w + 0.5f * u01(r.w));
    const float4 v = f.synth ? sv : xv;
    if (tid < 42) {  // 6 rows x 28 = 168 pixels = 42 groups of 4
      *reinterpret_cast<float4*>(xs + tid * 4) = v;
      const int row = d / 28;
      if (f.synth && row >= own_lo && row < own_hi) *reinterpret_cast<float4*>(f.x + b * 784 + d) = v;
    }
    if (f.synth && py == 0 && tid == 0) f.y[b] = label;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k)
    if (tid + 256 * k < 320) w1s[tid + 256 * k] = w1v[k];  // conv1 w [32][9] then b [32]
  lds_barrier();  // (the x rows / label just stored are read by later kernels only)
  MX_TRACE(f, 0, 1);
  // ---- stage 1b: conv1 + ReLU for 32 ci x 4 rows x 26 cols -> LDS tile, on MFMA: M = 104
  // positions (7 tiles of 16), N = 32 channels (2 tiles), K = 9 taps padded to 12 (3 k-steps).
  // Wave w owns N-tile (w & 1) and M-tiles (w >> 1) * 4 .. +3 (the last wave pair gets 3).
  {
    const int l16 = lane & 15, g = lane >> 4, nt = w & 1, mt0 = (w >> 1) * 4, mt1 = min(mt0 + 4, 7);
    const int ci_b = 16 * nt + l16;  // B column (channel) of this lane
    float bw[3];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int t = 4 * ks + g;
      bw[ks] = t < 9 ? w1s[ci_b * 9 + t] : 0.f;
    }
    for (int mt = mt0; mt < mt1; ++mt) {
      const int p = 16 * mt + l16, pr = p / 26, pc = p - pr * 26;  // A row (position) of this lane
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int t = 4 * ks + g, ky = t / 3, kx = t - 3 * ky;
        const float av = (t < 9 && p < 104) ? xs[(pr + ky) * 28 + pc + kx] : 0.f;
        c = mfma4(av, bw[ks], c);
      }
      // C: row = position 16 mt + 4g + j, column = channel 16 nt + l16
      const float bias = w1s[288 + ci_b];
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = 16 * mt + 4 * g + j;
        o[j] = fmaxf(c[j] + bias, 0.f);
        if (q < 104) {
          const int qr = q / 26, qc = q - qr * 26;
          tile[ci_b * kF2ChP + qr * kF2RowP + qc] = o[j];
        }
      }
      // publish the a1 rows this block owns (2, or 4 for the last row) for F6W straight from the
      // accumulators: the 4 rows of the strip are 104 contiguous floats of channel ci_b, so a
      // lane's 4 consecutive positions are one aligned float4 (no LDS read-back pass)
      const int q0 = 16 * mt + 4 * g;
      if (q0 < (py == 11 ? 104 : 52))
        st4(reinterpret_cast<float4*>(f.a1 + (size_t)b * 21632 + ci_b * 676 + row0 * 26 + q0),
            make_float4(o[0], o[1], o[2], o[3]), f.wt & 2);
    }
  }
  lds_barrier();  // the published a1 rows are read by F6W, not by this block
  MX_TRACE(f, 0, 2);
  f2_stage2_wino(f, sc, tile, b, py, w, lane);
  // side job of the first 8 blocks: this step's conv2 data-gradient Winograd filters for F7W
  if (blockIdx.x < 8) wino_dgrad_filter(f, sc, blockIdx.x * 256 + tid);
  MX_TRACE(f, 0, 5);
}

// ------------------------------------------------------------------------------------------
// F3: fc1 forward h_pre[b][n] = pool[b][:] . W1[n][:], output-tiled split-K on MFMA.
// Block = (K chunk of 1152, 16 x 16 output tile) -- 8 chunks x B/2 tiles (256 blocks at B = 64).
// Every block loads only its 16 pool rows and 16 W1 rows of the chunk (147 KB), and the tiles of
// one chunk sit on one XCD (xcd_remap), so that XCD's L2 holds the chunk's pool / W1 columns
// once.  Wave w of the 8 reduces K slice w of the chunk (144 deep, all 18 float4 operands issued
// up front, two accumulator chains), the 8 wave partials are summed in LDS in a fixed order, and
// one 64-bit fixed-point atomic per output per block adds the chunk partial into h (8 per
// output; integer adds, so h is exact and independent of the chunks' arrival order -- the float
// atomics this replaces made every step's rounding depend on it).  h was zeroed by the previous
// step's finalize.  (Measured alternatives, profiles/r3_mnist_knobs: 64-way split-K with 144-deep
// chunks 8.85 us; 16-way 576-deep chunks; 4 waves of 288-deep slices 7.8 us; this one 6.7 us.)
constexpr int kF3TChunks = 8, kF3TK = 9216 / kF3TChunks, kF3Wv = 8;
__global__ __launch_bounds__(64 * kF3Wv) void f3t_fc1_kernel(MnistFused f) {
  MX_TRACE(f, 1, 0);
  constexpr int kTW = kF3TK / kF3Wv, kTS = kTW / 16;
  // wave partials as [wave][j][64 lanes]: the stores (lane-linear) and the reads (thread = flat
  // index) are both bank-conflict free (the [16][17] row layout took 2-4 cycles per access)
  __shared__ float red[kF3Wv][4][64];
  const int tiles = f.B / 2;  // (B / 16) row tiles x 8 column tiles
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kc = bid / tiles, tile = bid - kc * tiles, mt = tile >> 3, nt = tile & 7;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const int k0 = kc * kF3TK + w * kTW + 4 * g;
  const float4* A = reinterpret_cast<const float4*>(f.pool + (size_t)(16 * mt + m) * 9216 + k0);
  const float4* W = reinterpret_cast<const float4*>(f.p + L::fw1 + (size_t)(16 * nt + m) * 9216 + k0);
  float4 av[kTS], bv[kTS];
#pragma unroll
  for (int s = 0; s < kTS; ++s) {
    av[s] = A[4 * s];
    bv[s] = W[4 * s];
  }
  // all 18 operand loads in flight before the first MFMA (left alone, the scheduler interleaves
  // each load with its MFMAs: 30 VGPRs, and the wave waits on memory once per k-step)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s = 0; s < kTS; ++s) {
    acc[0] = mfma4(av[s].x, bv[s].x, acc[0]);
    acc[1] = mfma4(av[s].y, bv[s].y, acc[1]);
    acc[0] = mfma4(av[s].z, bv[s].z, acc[0]);
    acc[1] = mfma4(av[s].w, bv[s].w, acc[1]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][j][lane] = acc[0][j] + acc[1][j];
  __syncthreads();
  if (tid < 256) {
    // flat index tid = (j, g, m): output row 4g + j, column m
    const int j = tid >> 6, l = tid & 63, row = 4 * (l >> 4) + j, col = l & 15;
    const float v = ((red[0][j][l] + red[1][j][l]) + (red[2][j][l] + red[3][j][l])) +
                    ((red[4][j][l] + red[5][j][l]) + (red[6][j][l] + red[7][j][l]));
    fix_add(f.h + (16 * mt + row) * 128 + 16 * nt + col, v, kHScale, carve(f.scratch, f.B).bad);
  }
  // F2 consumed the counter; bumped last so its load / wait does not hold wave 0 of block 0
  // in front of the operand loads
  if (f.synth && blockIdx.x == 0 && tid == 0) *f.counter += 1;
  MX_TRACE(f, 1, 1);
}

static void launch_f3(const MnistFused& f, hipStream_t st) {
  MX_LAUNCH(f3t_fc1_kernel, dim3(kF3TChunks * (f.B / 2)), dim3(64 * kF3Wv), 0, st, f);
}

// ------------------------------------------------------------------------------------------
// F5: head + fc1 backward for a 48-column slice of the 9216 fc1 inputs (192 blocks: at most one
// per CU, so no CU runs two of these latency-bound blocks back to back).
// Head (recomputed by EVERY block from the 32 KB h_pre; replaces a separate launch and its
// global dependency): h = ReLU(h_pre + b1); logits = h W2^T + b2 (MFMA, N = 10 padded to 16);
// log_softmax + NLL; argmax accuracy; dlogits = (softmax - onehot)/B; dh = (dlogits W2) *
// (h > 0) (MFMA, K = 10 padded to 16).  W2 lives in LDS transposed, w2t[n][c] (pitch 20,
// cols 10..15 zero), so both head GEMMs read it conflict-free.  The global side duties are
// spread so no block is much longer than the rest: blocks 0..9 store fc2 grad row c (+ bias
// grad c), block 10 the fc1 bias grad, block 0 the metrics.
// fc1: dW1[:, cols] = dh^T pool[:, cols] (M=128, K=B) and dp[:, cols] = dh W1[:, cols]
// (M=B, K=128), both on MFMA from LDS; dp is masked with the max-pool argmax / ReLU liveness
// (dead windows -> 0) and db2 accumulated (wave partials summed in order, one int64
// fixed-point add per block into the channel's accumulator).  dh lives in LDS as [B][132] (row pitch = 4 mod 32
// words: float4 row reads and 4-row-strided scalar reads are both bank-conflict free).
// LDS at B = 64: 92 KB (one block per CU by design).
// Up to 6 values held in NAMED registers across a long stretch of code: a plain array here
// (F5's prefetched fc1 operands, live across the head) was placed in scratch memory and re-read
// with dynamic offsets.  Accessed with compile-time k (inside fully unrolled loops).
template <typename T>
struct Reg6 {
  T r0, r1, r2, r3, r4, r5;
  __device__ __forceinline__ void set(int k, const T& x) {
    switch (k) {
      case 0: r0 = x; break;
      case 1: r1 = x; break;
      case 2: r2 = x; break;
      case 3: r3 = x; break;
      case 4: r4 = x; break;
      default: r5 = x; break;
    }
  }
  __device__ __forceinline__ T get(int k) const {
    switch (k) {
      case 0: return r0;
      case 1: return r1;
      case 2: return r2;
      case 3: return r3;
      case 4: return r4;
      default: return r5;
    }
  }
};

constexpr int kF5Cols = kFc1Cols, kF5NT = kF5Cols / 16, kF5C4 = kF5Cols / 4;
constexpr int kF5DhP = 132, kF5P = 52, kF5W2P = 20, kF5LgP = 20;  // kF5P = 4 mod 8: 4-row groups 16 banks apart
constexpr int kF5Misc = 12;  // [0..3] db2, [4..7] loss, [8..11] correct: one slot per wave
// Store of F5's bulk outputs (fc1 weights / momentum / dp): WT = agent-scope relaxed store
// (global_store ... sc1), which does not keep the line dirty in the XCD's L2, so the bytes drain
// to memory while the kernel still runs instead of in the end-of-kernel L2 write-back.
template <bool WT>
__device__ __forceinline__ void f5_store(float* p, float v) {
  if constexpr (WT)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
template <int B, bool WT, bool DEFER>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void f5_head_fc1_bwd_kernel(MnistFused f) {
  MX_TRACE(f, 2, 0);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dhs = sm;                       // [B][132]: h (post-ReLU), then dh in place
  float* ps = dhs + B * kF5DhP;          // [B][52]: pool columns of this slice
  float* wsm = ps + B * kF5P;            // [128][52]: W1 columns of this slice
  float* w2t = wsm + 128 * kF5P;         // [128][20]: W2^T, cols 10..15 zero
  float* lg = w2t + 128 * kF5W2P;        // [B][20]: logits, then dlogits (cols 10..15 zero)
  float* misc = lg + B * kF5LgP;         // [kF5Misc]: db2 / loss / correct partials per wave
  uint8_t* qs = reinterpret_cast<uint8_t*>(misc + kF5Misc);  // [B][48] argmax codes of this column slice
  const int c0 = blockIdx.x * kF5Cols;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  // folded fc1 SGD: this block owns weight columns c0..c0+47 of every row (old values in wsm);
  // the momentum of this thread's dW1 elements is loaded with the prologue's loads
  // Prologue in two groups so the head overlaps the fc1 operand loads: (1) the head's operands
  // (h, b1, W2, b2, labels) are loaded, staged and consumed first; (2) this slice's pool / argmax
  // / W1 (/ momentum) loads are issued right after group (1) and stay in flight (registers) while
  // the head runs -- the head has no global loads of its own, so its waits never drain them --
  // and are staged into LDS only after dh.  (Before: every load, then the head: ~3 us more.)
  constexpr int ND = B * 32 / 256, NP = (B * kF5C4 + 255) / 256, NW = (128 * kF5C4 + 255) / 256, N2 = 5;
  static_assert(NP <= 6 && NW <= 6, "F5 prefetch registers");
  longlong2 vd[ND][2];  // h_pre as int64 fixed point
  float4 vb1[ND];
  Reg6<float4> vp, vw;
  float v2[N2];
  Reg6<uint32_t> vq;  // argmax codes, 4 per uint32
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const int i = tid + 256 * k;
    const longlong2* hp = reinterpret_cast<const longlong2*>(f.h + (i >> 5) * 128 + (i & 31) * 4);
    vd[k][0] = hp[0];
    vd[k][1] = hp[1];
    vb1[k] = *reinterpret_cast<const float4*>(f.p + L::fb1 + (i & 31) * 4);
  }
#pragma unroll
  for (int k = 0; k < N2; ++k) v2[k] = f.p[L::fw2 + tid + 256 * k];  // 1280 = 5 x 256
  const int yv = f.y[tid < B ? tid : 0];
  const float b2v = f.p[L::fb2 + (m < 10 ? m : 0)];
  const int bad = *carve(f.scratch, f.B).bad;  // F3 saw a non-finite partial: h (and the loss) become NaN
  // group (2) strictly after group (1) in issue order: vmcnt counts in order, so a group-2 load
  // scheduled in front of a head operand would be waited for before the head
  __builtin_amdgcn_sched_barrier(0);
  // (2) fc1 operands: in flight during the head
  // folded fc1 SGD: this block owns weight columns c0..c0+47 of every row (old values in wsm);
  // the momentum of this thread's dW1 elements
  // (loaded unconditionally -- f.mom always exists: a load behind the fc1_sgd branch made the
  // waitcnt pass merge both paths and drain most of group 2 before the head)
  float mb[2][kF5NT][4];
  if constexpr (!DEFER) {  // DEFER: the update runs in F67's extra blocks, which load the momentum
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < kF5NT; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mb[a][c][j] = f.mom[L::fw1 + (size_t)(32 * w + 16 * a + 4 * g + j) * 9216 + c0 + 16 * c + m];
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int i = min(tid + 256 * k, B * kF5C4 - 1), r = i / kF5C4, c4 = i - r * kF5C4;
    if constexpr (!DEFER)  // the pool slice feeds only dW1
      vp.set(k, *reinterpret_cast<const float4*>(f.pool + (size_t)r * 9216 + c0 + c4 * 4));
    vq.set(k, *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(f.idx) + (size_t)r * 9216 + c0 +
                                                 c4 * 4));
  }
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int i = min(tid + 256 * k, 128 * kF5C4 - 1), r = i / kF5C4, c4 = i - r * kF5C4;
    vw.set(k, *reinterpret_cast<const float4*>(f.p + L::fw1 + (size_t)r * 9216 + c0 + c4 * 4));
  }
  // every group-2 load issued before the first head conversion: otherwise the scheduler hoists an
  // h fixed-point conversion above them and its wait delays all of group 2 by one load latency
  __builtin_amdgcn_sched_barrier(0);
  // (1) stage the head operands
#pragma unroll
  for (int k = 0; k < ND; ++k) {
    const int i = tid + 256 * k, c4 = (i & 31) * 4;
    const float4 b1 = vb1[k];
    const float4 hv = make_float4(from_fix_chk(vd[k][0].x, kHInv, bad), from_fix_chk(vd[k][0].y, kHInv, bad),
                                  from_fix_chk(vd[k][1].x, kHInv, bad), from_fix_chk(vd[k][1].y, kHInv, bad));
    *reinterpret_cast<float4*>(dhs + (i >> 5) * kF5DhP + c4) =
        make_float4(relu_nan(hv.x + b1.x), relu_nan(hv.y + b1.y), relu_nan(hv.z + b1.z), relu_nan(hv.w + b1.w));
  }
#pragma unroll
  for (int k = 0; k < N2; ++k) {
    const int i = tid + 256 * k;
    w2t[(i & 127) * kF5W2P + (i >> 7)] = v2[k];
  }
  for (int i = tid; i < 128 * 6; i += 256) w2t[(i / 6) * kF5W2P + 10 + i % 6] = 0.f;
  if (tid < kF5Misc) misc[tid] = 0.f;
  __syncthreads();
  MX_TRACE(f, 2, 1);
  // ---- head: logits (wave w: batch M-tiles w, w+4, ...; K = 128 permuted for float4 A reads)
  for (int mt = w; mt < B / 16; mt += 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* arow = dhs + (16 * mt + m) * kF5DhP + 4 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 av = *reinterpret_cast<const float4*>(arow + 16 * s);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma4(sel4(av, j), w2t[(16 * s + 4 * g + j) * kF5W2P + m], acc);
    }
    if (m < 10) {
#pragma unroll
      for (int j = 0; j < 4; ++j) lg[(16 * mt + 4 * g + j) * kF5LgP + m] = acc[j] + b2v;
    }
  }
  __syncthreads();
  MX_TRACE(f, 2, 2);
  // ---- head: softmax / NLL / accuracy / dlogits (one thread per row)
  float loss_v = 0.f, corr_v = 0.f;
  if (tid < B) {
    // rows f.nB.. pad the last 16-row tile (batch not a multiple of 16): no loss, no accuracy,
    // zero dlogits -- so they add nothing to any gradient downstream
    const float live = tid < f.nB ? 1.f : 0.f;
    float* l = lg + tid * kF5LgP;
    float mx = l[0];
    int am = 0;
#pragma unroll
    for (int c = 1; c < 10; ++c)
      if (l[c] > mx) { mx = l[c]; am = c; }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) se += __expf(l[c] - mx);
    const float lse = mx + __logf(se);
    const int y = yv;
    float ly = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) ly = c == y ? l[c] : ly;
    loss_v = (lse - ly) * live;
    corr_v = am == y ? live : 0.f;
    const float inv = live / (float)f.nB;
#pragma unroll
    for (int c = 0; c < 10; ++c) l[c] = (__expf(l[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
#pragma unroll
    for (int c = 10; c < 16; ++c) l[c] = 0.f;
  }
  if (blockIdx.x == 0 && 64 * w < B) {  // batch loss / correct: one slot per wave
    const float ls = wave_sum(loss_v), cs = wave_sum(corr_v);
    if (lane == 0) {
      misc[4 + w] = ls;
      misc[8 + w] = cs;
    }
  }
  __syncthreads();
  MX_TRACE(f, 2, 3);
  if (blockIdx.x < 10 && tid <= 128) {  // fc2 grad row c = blockIdx.x (+ its bias grad) from h and dlogits
    // 8 independent partial sums (B % 16 == 0): no serial LDS-latency chain, so blocks 0..9
    // finish with the rest of the grid
    const int c = blockIdx.x;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (tid < 128) {
      for (int b = 0; b < B; b += 8)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(lg[(b + k) * kF5LgP + c], dhs[(b + k) * kF5DhP + tid], acc[k]);
    } else {
      for (int b = 0; b < B; b += 8)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += lg[(b + k) * kF5LgP + c];
    }
    const float sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    f.g[tid < 128 ? L::fw2 + c * 128 + tid : L::fb2 + c] = sum;
  }
  if (blockIdx.x == 0 && tid == 0 && f.metrics) {
    atomicAdd(f.metrics, (misc[4] + misc[5]) + (misc[6] + misc[7]));
    atomicAdd(f.metrics + 1, (misc[8] + misc[9]) + (misc[10] + misc[11]));
  }
  if (blockIdx.x < 10) __syncthreads();  // the fc2 grad read h before dh overwrites it
  // ---- head: dh = (dlogits W2) * (h > 0), in place over h (K = 16: c 10..15 are zero)
  for (int mt = w; mt < B / 16; mt += 4) {
    const float4 av = *reinterpret_cast<const float4*>(lg + (16 * mt + m) * kF5LgP + 4 * g);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const float4 bv = *reinterpret_cast<const float4*>(w2t + (16 * nt + m) * kF5W2P + 4 * g);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = mfma4(av.x, bv.x, acc);
      acc = mfma4(av.y, bv.y, acc);
      acc = mfma4(av.z, bv.z, acc);
      acc = mfma4(av.w, bv.w, acc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float* d = dhs + (16 * mt + 4 * g + j) * kF5DhP + 16 * nt + m;
        *d = *d > 0.f ? acc[j] : 0.f;
      }
    }
  }
  // (2) stage the fc1 operands (their loads have been in flight since the prologue)
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int i = tid + 256 * k, r = i / kF5C4, c4 = i - r * kF5C4;
    if (i < B * kF5C4) {
      if constexpr (!DEFER) *reinterpret_cast<float4*>(ps + r * kF5P + c4 * 4) = vp.get(k);
      *reinterpret_cast<uint32_t*>(qs + r * kF5Cols + c4 * 4) = vq.get(k);
    }
  }
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int i = tid + 256 * k, r = i / kF5C4, c4 = i - r * kF5C4;
    if (i < 128 * kF5C4) *reinterpret_cast<float4*>(wsm + r * kF5P + c4 * 4) = vw.get(k);
  }
  __syncthreads();
  MX_TRACE(f, 2, 4);
  if (blockIdx.x == 10 && tid < 128) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; b += 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += dhs[(b + k) * kF5DhP + tid];
    f.g[L::fb1 + tid] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
  if constexpr (DEFER) {  // publish dh for the deferred update: blocks 0 .. B/8-1 write 8 rows each
    if ((int)blockIdx.x < B / 8) {
      const int r = 8 * (int)blockIdx.x + (tid >> 5), c4 = (tid & 31) * 4;
      *reinterpret_cast<float4*>(f.dh + r * 128 + c4) = *reinterpret_cast<const float4*>(dhs + r * kF5DhP + c4);
    }
  }
  // ---- dW1 tiles: rows n (8 M-tiles, wave w takes 2w, 2w+1), cols kF5NT N-tiles, K = B
  if constexpr (!DEFER) {
    f32x4 acc[2][kF5NT];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < kF5NT; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < B / 16; ++s) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = 16 * s + 4 * g + j;
        const float a0 = dhs[b * kF5DhP + 32 * w + m], a1v = dhs[b * kF5DhP + 32 * w + 16 + m];
#pragma unroll
        for (int c = 0; c < kF5NT; ++c) {
          const float bv = ps[b * kF5P + 16 * c + m];
          acc[0][c] = mfma4(a0, bv, acc[0][c]);
          acc[1][c] = mfma4(a1v, bv, acc[1][c]);
        }
      }
    }
    if (!f.fc1_sgd) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < kF5NT; ++c)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = 32 * w + 16 * a + 4 * g + j;
            f5_store<WT>(f.g + L::fw1 + (size_t)n * 9216 + c0 + 16 * c + m, acc[a][c][j]);
          }
    } else {  // the gradient is consumed here (not materialised in g)  // the SGD kernel's update, same operation order (gscale = 1: world size 1)
      const float lr = *f.lr;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < kF5NT; ++c)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = 32 * w + 16 * a + 4 * g + j;
            const size_t e = L::fw1 + (size_t)n * 9216 + c0 + 16 * c + m;
            float pv = wsm[n * kF5P + 16 * c + m], bv = mb[a][c][j];
            sgd_upd(pv, bv, acc[a][c][j], 1.f, f.sgd_mom, f.sgd_wd, lr);
            f5_store<WT>(f.mom + e, bv);
            f5_store<WT>(f.p + e, pv);
          }
    }
  }
  MX_TRACE(f, 2, 5);
  // ---- dp tiles: rows b (M-tiles of 16, wave-strided), cols kF5NT N-tiles, K = 128.  The 48
  // columns of a slice never straddle a conv2 channel (144 = 3 x 48), so db2 has one target.
  float db2_part = 0.f;
  for (int mt = w; mt < B / 16; mt += 4) {
    f32x4 acc[kF5NT];
#pragma unroll
    for (int c = 0; c < kF5NT; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* arow = dhs + (16 * mt + m) * kF5DhP + 4 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 av = *reinterpret_cast<const float4*>(arow + 16 * s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * s + 4 * g + j;
#pragma unroll
        for (int c = 0; c < kF5NT; ++c) acc[c] = mfma4(sel4(av, j), wsm[n * kF5P + 16 * c + m], acc[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < kF5NT; ++c) {
      const int kk = c0 + 16 * c + m;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = 16 * mt + 4 * g + j;
        const bool alive = qs[b * kF5Cols + 16 * c + m] < 4;
        const float v = alive ? acc[c][j] : 0.f;
        f5_store<WT>(f.dp + (size_t)b * 9216 + kk, v);
        db2_part += v;
      }
    }
  }
  {
    const float s = wave_sum(db2_part);
    if (lane == 0) misc[w] = s;
  }
  __syncthreads();
  MX_TRACE(f, 2, 6);
  if (tid == 0) {
    const Scratch sc = carve(f.scratch, f.B);
    fix_add(sc.db2 + c0 / 144, (misc[0] + misc[1]) + (misc[2] + misc[3]), kGScale, sc.bad);
  }
  MX_TRACE(f, 2, 7);
}

// ------------------------------------------------------------------------------------------
// SGD over the flat parameter buffer (PyTorch semantics; DDP's 1/world_size folded into
// gscale) + repack of the updated conv2 weights into F2's Winograd fragment order.
// kFin (no gradient collectives in the step, i.e. world size 1): F8's duties are folded in --
// the conv2 weight grad is summed from the per-image slabs, the conv1 and conv2-bias grads are
// converted from their int64 fixed-point accumulators, all of them are reset (and written to g
// for inspection), and h is zeroed -- one launch and one kernel boundary fewer per step.
template <bool kFin>
__global__ __launch_bounds__(256) void sgd_pack_kernel(MnistFused f, Scratch sc, float* __restrict__ buf,
                                                       const float* __restrict__ lr_ptr, float gscale, float mom,
                                                       float wd) {
  const float lr = *lr_ptr;
  // kFin: the last kWslabGroups blocks sum the conv2 weight-gradient slabs (4 (co, ci) pairs
  // each, fixed order) and update + repack those pairs; the other nflat blocks do the rest
  const int ngrp = kFin ? kWslabGroups : 0, nflat = (int)gridDim.x - ngrp;
  if ((int)blockIdx.x >= nflat) {
    __shared__ float red[576 + 36];
    const int grp = (int)blockIdx.x - nflat;
    // the pair's weights / momentum are requested before the slab sum (one round trip for both)
    const int pair = 4 * grp + min((int)threadIdx.x, 3), e0 = (int)L::w2 + pair * 9;
    float pe[9], bb[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      pe[r] = f.p[e0 + r];
      bb[r] = buf[e0 + r];
    }
    wslab_group_sum(f, sc, grp, red, red + 576);
    if (threadIdx.x < 4) {
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        const float gg = red[576 + 9 * threadIdx.x + r];
        sgd_upd(pe[r], bb[r], gg, gscale, mom, wd, lr);
        f.g[e0 + r] = gg;
        buf[e0 + r] = bb[r];
        f.p[e0 + r] = pe[r];
      }
      conv2_pack_pair(sc, pair, pe);
    }
    return;
  }
  float4* p4 = reinterpret_cast<float4*>(f.p);
  float4* g4 = reinterpret_cast<float4*>(f.g);
  float4* b4 = reinterpret_cast<float4*>(buf);
  constexpr int n4 = (int)(L::total / 4);  // 299970 float4 (total = 1199882 = 4*299970 + 2)
  if (kFin) {
    longlong2* h2 = reinterpret_cast<longlong2*>(f.h);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < f.B * 64; i += nflat * 256) h2[i] = make_longlong2(0, 0);
  }
  constexpr int kW2a = (int)L::w2 / 4, kW2b = ((int)L::w2 + kPack) / 4;  // conv2 weights (float4 range)
  constexpr int kF1a = (int)L::fw1 / 4, kF1n = ((int)L::fb1 - (int)L::fw1) / 4;  // fc1 weights (float4 range)
  static_assert(L::fw1 % 4 == 0 && L::fb1 % 4 == 0 && L::b2 % 4 == 0, "fc1 / conv2 bias must be float4-aligned");
  const int skip = f.fc1_sgd ? kF1n : 0;  // fc1 updated by F5: iterate around it
  for (int t = blockIdx.x * 256 + threadIdx.x; t < n4 - skip; t += nflat * 256) {
    const int i = t >= kF1a ? t + skip : t;
    if (i >= kW2a && i < kW2b) continue;  // per (co, ci) pair below
    float4 pv = p4[i];
    float4 gv = g4[i];
    if (kFin && (i < kW2a || (i >= kW2b && i < kW2b + 16))) {
      // conv1 w/b: exact int64 sum of the slabs; conv2 bias: its accumulator.  Then reset them.
      long long a[4] = {0, 0, 0, 0};
      if (i < kW2a) {
        longlong2* sl = reinterpret_cast<longlong2*>(sc.g1) + 2 * i;
#pragma unroll
        for (int k0 = 0; k0 < kG1Slabs; k0 += 8) {
          longlong2 v[16];  // 8 slabs' loads in flight, then the adds
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            v[2 * k] = sl[(k0 + k) * 160];
            v[2 * k + 1] = sl[(k0 + k) * 160 + 1];
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            a[0] += v[2 * k].x;
            a[1] += v[2 * k].y;
            a[2] += v[2 * k + 1].x;
            a[3] += v[2 * k + 1].y;
          }
        }
#pragma unroll
        for (int k = 0; k < kG1Slabs; ++k) {
          sl[k * 160] = make_longlong2(0, 0);
          sl[k * 160 + 1] = make_longlong2(0, 0);
        }
      } else {
        longlong2* d = reinterpret_cast<longlong2*>(sc.db2) + 2 * (i - kW2b);
        const longlong2 v0 = d[0], v1 = d[1];
        a[0] = v0.x;
        a[1] = v0.y;
        a[2] = v1.x;
        a[3] = v1.y;
        d[0] = make_longlong2(0, 0);
        d[1] = make_longlong2(0, 0);
      }
      const int bad = *sc.bad;
      gv = make_float4(from_fix_chk(a[0], kGInv, bad), from_fix_chk(a[1], kGInv, bad), from_fix_chk(a[2], kGInv, bad),
                       from_fix_chk(a[3], kGInv, bad));
      g4[i] = gv;
    }
    float4 bv = b4[i];
    sgd_upd(pv.x, bv.x, gv.x, gscale, mom, wd, lr);
    sgd_upd(pv.y, bv.y, gv.y, gscale, mom, wd, lr);
    sgd_upd(pv.z, bv.z, gv.z, gscale, mom, wd, lr);
    sgd_upd(pv.w, bv.w, gv.w, gscale, mom, wd, lr);
    b4[i] = bv;
    p4[i] = pv;
  }
  // !kFin (the gradient was all-reduced, F8 wrote it to g): conv2 weights, one thread per
  // (co, ci) pair updates its 9 taps and rewrites its Winograd filter.  The pairs go to wave 0
  // of the grid's last 32 blocks (one main-loop pass each: 32 CUs share the scattered stores);
  // all 27 loads are issued before any store.
  const int pair = ((int)blockIdx.x - (nflat - 32)) * 64 + (int)threadIdx.x;
  if (!kFin && (int)blockIdx.x + 32 >= nflat && threadIdx.x < 64 && pair >= 0 && pair < 2048) {
    const int e0 = (int)L::w2 + pair * 9;
    float gg[9], pe[9], bb[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      gg[r] = f.g[e0 + r];
      pe[r] = f.p[e0 + r];
      bb[r] = buf[e0 + r];
    }
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      sgd_upd(pe[r], bb[r], gg[r], gscale, mom, wd, lr);
      buf[e0 + r] = bb[r];
      f.p[e0 + r] = pe[r];
    }
    conv2_pack_pair(sc, pair, pe);
  }
  if (blockIdx.x == 0 && threadIdx.x < (int)(L::total - 4 * n4)) {  // 2-element tail (fc2.bias)
    const int e = 4 * n4 + threadIdx.x;
    float pe = f.p[e], bb = buf[e];
    sgd_upd(pe, bb, f.g[e], gscale, mom, wd, lr);
    buf[e] = bb;
    f.p[e] = pe;
  }
}

}  // namespace
}  // namespace mnist

using namespace mnist;

size_t mnist_fused_scratch_floats(int B) { return scratch_floats(B); }

// default: F5, F2 and F6W.  Round 4 measured F2 + F6W +0.9 % and F5's own stores -0.7 %
// (profiles/r4_ab*); with round 5's F6W / F3 the F5 stores pay too: 936-938k vs 928-930k img/s at
// the driver's length, 940-942k vs 933-935k at 2,000 steps (profiles/r5_wt/)
static int g_wt_stores = 7;
void mnist_set_wt_stores(int mask) { g_wt_stores = mask & 7; }
int mnist_wt_stores() { return g_wt_stores; }


static void check(const MnistFused& f) {
  MX_CHECK(f.B % 16 == 0 && f.B >= 16 && f.B <= 128 && f.nB >= 1 && f.nB <= f.B && f.B - f.nB < 16,
           "fused MNIST engine: 1 <= batch <= 128, buffers padded to the next multiple of 16");
}

static void set_lds_limits() {
  static bool done = false;
  if (done) return;
#define F5_FN(b) reinterpret_cast<const void*>(f5_head_fc1_bwd_kernel<b, false, false>), \
                reinterpret_cast<const void*>(f5_head_fc1_bwd_kernel<b, true, false>), \
                reinterpret_cast<const void*>(f5_head_fc1_bwd_kernel<b, false, true>), \
                reinterpret_cast<const void*>(f5_head_fc1_bwd_kernel<b, true, true>)
  const void* fns[] = {F5_FN(16), F5_FN(32), F5_FN(48), F5_FN(64), F5_FN(80), F5_FN(96), F5_FN(112), F5_FN(128)};
#undef F5_FN
  for (const void* fn : fns)
    MX_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  done = true;
}

void mnist_fused_init(const MnistFused& f, hipStream_t st) {
  check(f);
  set_lds_limits();
  MX_LAUNCH(k_init, dim3(128), dim3(256), 0, st, f, carve(f.scratch, f.B));
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_forward(const MnistFused& f, hipStream_t st) {
  check(f);
  set_lds_limits();
  const Scratch sc = carve(f.scratch, f.B);
  MX_LAUNCH(f2_fwd_kernel, dim3(f.B * 12), dim3(256), 0, st, f, sc);
  launch_f3(f, st);
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_fc1_bwd(const MnistFused& f, hipStream_t st) {
  const size_t lds = sizeof(float) * ((size_t)f.B * kF5DhP + f.B * kF5P + 128 * kF5P + 128 * kF5W2P + f.B * kF5LgP + kF5Misc) +
                     (size_t)f.B * kF5Cols;
  const dim3 grid(9216 / kF5Cols), block(256);
  const bool defer = f.fc1_defer != 0;
  void (*kfn)(MnistFused) = nullptr;
#define F5_CASE(b)                                                                                           \
  case b:                                                                                                    \
    if (defer) kfn = (f.wt & 1) ? f5_head_fc1_bwd_kernel<b, true, true> : f5_head_fc1_bwd_kernel<b, false, true>; \
    else kfn = (f.wt & 1) ? f5_head_fc1_bwd_kernel<b, true, false> : f5_head_fc1_bwd_kernel<b, false, false>;   \
    break;
  switch (f.B) {
    F5_CASE(16) F5_CASE(32) F5_CASE(48) F5_CASE(64) F5_CASE(80) F5_CASE(96) F5_CASE(112) F5_CASE(128)
    default: MX_CHECK(false, "unsupported fused batch");
  }
#undef F5_CASE
  MX_LAUNCH(kfn, grid, block, lds, st, f);
  MX_HIP_CHECK(hipGetLastError());
}

// 2 (default): MNIST driver length 933-938k -> 979-980k img/s, 2,000 steps 938k -> 985k
// (profiles/r6_fc1defer/); 1 measured 926-930k vs 931-936k (profiles/r6_f67defer/)
static int g_fc1_defer = 2;
void mnist_set_fc1_defer(int mode) { g_fc1_defer = mode < 0 ? 0 : (mode > 2 ? 2 : mode); }
int mnist_fc1_defer() { return g_fc1_defer; }

void mnist_fused_sgd(const MnistFused& f, float* mom_buf, const float* lr, float gscale, float momentum, float wd,
                     hipStream_t st, bool finalize) {
  MX_CHECK(!f.fc1_sgd || (finalize && gscale == 1.f && f.mom == mom_buf),
           "fc1 SGD is folded into F5 only without gradient collectives");
  // folded: ~20 K elements left (+ the 32 pair blocks, or the 512 slab-sum pair-group blocks)
  const dim3 grid((f.fc1_sgd ? 128 : 1024) + (finalize ? kWslabGroups : 0));
  if (finalize)
    MX_LAUNCH(sgd_pack_kernel<true>, grid, dim3(256), 0, st, f, carve(f.scratch, f.B), mom_buf, lr, gscale, momentum, wd);
  else
    MX_LAUNCH(sgd_pack_kernel<false>, grid, dim3(256), 0, st, f, carve(f.scratch, f.B), mom_buf, lr, gscale, momentum, wd);
  MX_HIP_CHECK(hipGetLastError());
}

}  // namespace mx

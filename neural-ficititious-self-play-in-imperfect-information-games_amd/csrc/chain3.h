// The SGD chain kernel (k_chain3) and its helpers, shared by the two translation units that
// instantiate it: learner.hip (BR, k_chain3<1, *>) and chain_ar.hip (AR, k_chain3<0, *>).
// The two are compiled with different scheduler flags (__graft_entry__.FILE_FLAGS).
#pragma once
#include <atomic>
#include <type_traits>

#include "engine_internal.h"

namespace nfsp {
namespace chain {
namespace nn = nfsp::nn;
using namespace nfsp::eng;

// ---------------------------------------------------------------------------
// SGD chains: one workgroup (4 waves) per (agent, net) runs that net's updates back to
// back with the whole net in registers (k_chain3).  Reference: agent/agent.py:241-264
// (model.fit(batch_size=32, epochs=2) of the BR Q-net and the AR policy net).
// ---------------------------------------------------------------------------
// One chain workgroup's work: a net's weights and the step records of one (engine, agent).
struct ChainJob {
  float* w;                       // weights of (agent, net)
  float* sync_to;                 // BR: target net to copy into at the end (or null)
  float* snap_to;                 // a pipelined slice's snapshot of the net (or null)
  const StepRec* rec;             // this agent's step records [umax][E][B / 32] (prep kernels)
  const uint8_t* active;          // AR: per-update flag, 0..0 1..1 in u (null for BR)
  float* loss_out;                // optional: [umax][E] Keras epoch losses (the values the
                                  // reference's TensorBoard callbacks log, agent/agent.py:84-88)
  int64_t u0, u1;                 // update range
};
struct ChainArgs {
  ChainJob job[2];                // blockIdx -> job (one engine: <= 2 workgroups)
  const ChainJob* jobs;           // device table instead, when set (engine groups: 2R workgroups)
  int B, E;
  unsigned long long* stamps;     // diagnostic build only (NFSP_CHAIN_STAMPS): phase cycles
  int lds;                        // host side: dynamic LDS per workgroup (0: CHAIN_LDS, a CU
                                  // to itself; engine groups of > 64 replicas share CUs)
};

// In-kernel phase stamps (cdna_hip_programming.md §7): a separate diagnostic build only.
#ifdef NFSP_CHAIN_STAMPS
#define CHAIN_STAMP(k)                                                                   \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long _t;                                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");          \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    st_acc[k] += _t - st_last;                                                          \
    st_last = _t;                                                                       \
  } while (0)
#else
#define CHAIN_STAMP(k) do { } while (0)
#endif

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
// A 16-byte LDS read of which 12 bytes are used.  Through HIP's float4 the compiler narrows
// it to ds_read_b96, which takes 8 LDS cycles per wave instead of ds_read_b128's 4
// (MI355X_MICROARCH.md, LDS table); through the vector type it stays ds_read_b128.
__device__ inline floatx4 lds4(const void* p) { return *reinterpret_cast<const floatx4*>(p); }
// The same, volatile (through an LDS pointer: a generic volatile pointer becomes a flat load):
// a read whose first two components feed packed f32 instructions is otherwise still narrowed
// to ds_read_b96.
typedef __attribute__((address_space(3))) const volatile floatx4 lds_vfloatx4;
__device__ inline floatx4 lds4v(const void* p) { return *(lds_vfloatx4*)p; }

// Packed f32 (v_pk_fma_f32 / v_pk_mul_f32: two values per instruction, each half rounded
// exactly as the scalar instruction) where a step has pairs of independent scalar operations
// (round 4, tools/ar_var.sh; weight hashes after 400 updates identical to the scalar chain):
//   PK_W   the W1 update (8 fma -> 4), both chains
//   PK_SM  AR softmax: y = e / S and d = y T_M - m for outputs 0 / 1
//   PK_L2  layer 2: the two sample halves' partial outputs (24 fma -> 12)
//   PK_O   outputs 0 / 1 of the 4-wave partial sums (8 add -> 4)
// Kept: BR PK_W, AR PK_W | PK_SM (AR 0.788 -> 0.761 us per SGD step in the microbenchmark).
// Not kept, because their results were not reproducible:
//  * PK_L2 in the AR chain (whose Z1 MFMAs are scheduled freely, see the fences in the
//    step): the weights differed on every run (4e-3 .. 9e-3 from the f32 reference chain
//    after 200 updates); in that schedule a packed FMA overwrote the SrcC registers of a
//    dependent MFMA 2-3 wait states after it issued;
//  * PK_L2 / PK_O in the BR chain: bit-identical and 0.750 -> 0.712 us with a CU per chain,
//    but with 4 chain workgroups per CU (engine groups of 200 replicas,
//    tests/test_gpu_group.py) replicas differed from standalone engines by up to 3e-4 on
//    some runs (tools/group_share_probe.py).  Their schedules overwrite the SrcC or result
//    registers of in-flight MFMAs by VALU instructions 4-7 wait states after issue 16 times
//    per step, against 4 in the scalar chain: the compiler's MFMA hazard padding is not
//    enough there when other waves share the matrix cores.  Every kept variant was checked
//    with that probe (R = 200, exact) as well as the GPU parity suite.
//  * also measured: PK_O in the AR chain (0.772, slower), the BR Huber loss on pairs (0.737).
constexpr unsigned PK_L2 = 1, PK_O = 2, PK_W = 4, PK_SM = 8;
#ifndef NFSP_PK_AR                 // build-time override, for A/B builds (tools/build_lib_variant.py)
#define NFSP_PK_AR (PK_W | PK_SM)
#endif
#ifndef NFSP_PK_BR
#define NFSP_PK_BR (PK_W)
#endif
template <int RELU>
constexpr unsigned chain_pk() { return RELU == 0 ? (NFSP_PK_AR) : (NFSP_PK_BR); }
// NFSP_CHAIN_G0ROW: gb2[0] enters the V transpose as each lane row's 16-sample sum instead of
// the 32-sample total (see own1_sc).  Measured in round 6 and left off: tools/r06.sh chain_ab
// gave AR 0.760 -> 0.750 us per SGD step but BR 0.721 -> 0.727; built into the AR chain only,
// the driver's bench read 7.02M hands/s (7.09M without) and the Leduc learner parity case with
// the textbook extensions (quirks 120) moved to 2.1e-3 against its 1e-3 bound (a ReLU crossing
// follows the new summation order).  Also measured and dropped: the BR loss without relu(o)
// in e and with -1 / (3 x batch) folded into the rate, 5 instructions fewer per step but
// 0.721 -> 0.736 (the schedule moved).
#ifndef NFSP_CHAIN_G0ROW
#define NFSP_CHAIN_G0ROW 0
#endif

__device__ inline float dpp_f(float x, int ctrl) {
  switch (ctrl) {   // the control word must be an immediate
    case 0x128: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
    case 0xB1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
    case 0x4E: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));
  }
}

__device__ inline float dpp_any(float x, int ctrl) {
  switch (ctrl) {
    case 0x121: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xF, 0xF, false));
    case 0x122: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xF, 0xF, false));
    case 0x124: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));
    default: return dpp_f(x, ctrl);
  }
}

// x + partner(lane ^ 32) in every lane
__device__ inline float sum_x32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// x + partner(lane ^ 16) in every lane
__device__ inline float sum_x16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Sums over the 32 samples held by the loss lanes (k_chain3's `ls` layout: every sample in 2
// lanes), in every lane, added in exactly the round-3 chain's order (it held sample c in lane
// c of rows 0 / 1 and 16 + c in rows 2 / 3, summed each row by DPP row_ror 8, 4, 2, 1, then
// the two halves): pairs s, s ^ 8 (rows g, g ^ 2), s ^ 4 (lanes c, c ^ 8), s ^ 2, s ^ 1 (quad
// permutes), then samples 0-15 + 16-31 (lanes c, c ^ 4).  a + b == b + a bit for bit, so
// every level is the round-3 level, and the 32-sample totals are bit-identical to it.
template <int CTRL>
__device__ inline float dpp_bc(float x) {           // every lane has a source: bound_ctrl on
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, true));
}
__device__ inline float tot_rows(float x) {        // levels 2 .. 5, after the rows' level 1
  x = x + dpp_bc<0x128>(x);
  x = x + dpp_bc<0x4E>(x);
  x = x + dpp_bc<0xB1>(x);
  return x + dpp_bc<0x124>(x);
}
__device__ inline float tot32(float x) { return tot_rows(sum_x32(x)); }
// two totals at once: rows 0 / 1 get a's, rows 2 / 3 b's
__device__ inline float tot32_pair(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return tot_rows(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}

// ---------------------------------------------------------------------------
// k_chain3: the SGD chain on bf16 matrix cores with exact-f32 operands.
//
// An f32 value v is split exactly into three bf16 terms v = hi + mid + lo (8 + 8 + 8
// significand bits, round-to-nearest at each cut), and a Leduc observation is 0/1, so
// X.W = X.lo + X.mid + X.hi with every product exact and f32 accumulation: the 16 chained
// v_mfma_f32_16x16x4_f32 of a layer-1 product become 3 v_mfma_f32_16x16x32_bf16 per tile
// (K = 32 covers all 30 inputs).  Per wave (hidden slice 16w..16w+15, lane (g, c) =
// (l >> 4, l & 15)):
//   * layer-1 K slot 8g + j <-> input pi(g, j) = 4g + j (j < 4) or 16 + 4g + j - 4, so the
//     dW1 accumulator lands in the registers that hold W1 (wr[j] = W1[pi(g, j)][16w + c]).
//     Input 30 is the constant 1 (CHAIN_BIAS_BIT).  Its row holds b1, so the layer-1
//     products include the bias, and dW1's row 30 is gb1;
//   * forward twice from the same registers: Z1 sample-major (D row = sample, for the
//     backward and dW1) and Z1^T hidden-major (D row = hidden: layer 2 is then 4 lane-local
//     FMAs per output plus two permlane swaps instead of a 16-lane reduction);
//   * dW1 = X^T dZ1 with K = samples (K slot 8g + j <-> sample 16 (j >> 2) + 4g + (j & 3));
//   * every bit operand comes ready-made from the step record (StepRec: the prep kernels
//     expand the masks to bf16 0/1 fragments).  Records pass through a 4-slot LDS ring:
//     each wave loads a quarter of record t + 2 during step t, and step t + 1's barrier
//     publishes it.  The dW1 operand X^T is the same fa image read transposed
//     (ds_read_b64_tr_b16), so a record is the fa image and the targets, 2,560 B;
//   * one barrier per step (the 4 waves' layer-2 partials); all other exchange is
//     wave-private (LDS w2t) or cross-lane (DPP, permlane).  The loss gradients reach the
//     backward's sample-major layout by DPP row broadcasts fused into its FMAs (bwd_dpp).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifdef NFSP_CHAIN_STAMPS
// diagnostic build: [RELU * 2 + block][wave][phase 0-5, -, -, kernel cycles, steps] for the
// one-engine launches (blocks 0, 1); table launches (engine groups) are not stamped
static __device__ unsigned long long g_chain_stamps[8][4][10];
#endif

// Stores are unconditional: lanes whose copy is redundant (the rows g > 0 of w2t, the lanes
// past a record quarter) write to sink rows nobody reads, so the loop has no exec-mask
// branches.
struct Chain3Smem {
  float po[2][4][64][4];     // per-wave partial layer-2 outputs by sample (rows 0..31 used),
                             // double-buffered by step parity
  float4 w2t[4][64];         // wave-private: W2[h][0..2] of the slice (rows 0..15: the layer-2
                             // weights live here, each component written by the lanes owning it)
  float b2s[4][4];           // wave-private: b2
  StepRec ring[4];           // step records t .. t + 2 (slot t & 3), a quarter per wave
  uint4 rec_sink[64];
};
constexpr int REC_CHUNKS = (int)(sizeof(StepRec) / 16);    // 160 x 16 B
constexpr int REC_QUARTER = REC_CHUNKS / 4;                 // 40 per wave: one chunk per lane
static_assert(REC_CHUNKS % 4 == 0 && REC_QUARTER <= 64, "record chunking");
// Reserve (nearly) all of a CU's LDS for a chain workgroup: a chain then has its CU to
// itself -- no prep / target kernel's waves share its SIMDs.
constexpr int CHAIN_LDS = 150 * 1024;
static_assert(sizeof(Chain3Smem) <= CHAIN_LDS, "chain LDS");
// LDS per chain workgroup when `per_cu` of them must be resident on a CU at once (engine
// groups with more chain workgroups than CUs): an equal share of the CU's 160 KB
inline int chain_lds_shared(int per_cu) {
  if (per_cu <= 1) return CHAIN_LDS;
  const int share = (160 * 1024 / per_cu) & ~1023;
  return share - 1024 >= (int)sizeof(Chain3Smem) ? share - 1024 : (int)sizeof(Chain3Smem);
}

// exact three-term bf16 split of 8 f32 values, a pair at a time: per pair and level one
// packed conversion (v_cvt_pk_bf16_f32, round to nearest even) and the two residuals by a
// bf16 dot: a - hi(a) = dot((hi(a), hi(b)), (-1, 0)) + a, exact (the product is exact and the
// difference is representable).  v = hi + mid + lo exactly.  7 instructions per pair instead
// of 11 (a shift / mask and a subtract per residual).  History (tools/chain_ab.sh, results
// bit-identical throughout): the builtin's accumulating v_dot2c_f32_bf16 took BR 0.906 ->
// 0.884 us, AR 0.93 -> 0.923 us per SGD step; the asm form below saves its v_movs (0.885 ->
// 0.877 / 0.930 -> 0.921).  Details:
//  * the (-1, 0) / (0, -1) operands come from VGPRs made once per kernel: written as the
//    literal 0x0000bf80 the pair did not reach the instruction as given;
//  * an asm conversion next to compiler-placed dot2c moved the chain's results (up to 2e-3
//    after 200 updates): gfx950 needs wait states between a DOT write and another VALU
//    instruction's read, and the compiler pads only for instructions it can see.  So the
//    whole split is ONE asm statement that spaces them itself.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ inline uint32_t cvt_pk_bf16(float a, float b) {
  const bf16x2 r = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, r);
}
// the (-1, 0) / (0, -1) bf16 pairs of the residual dots, made once per kernel
struct SplitK {
  uint32_t cl, ch;
};
__device__ inline SplitK split_consts() {
  SplitK k;
  asm volatile("v_mov_b32 %0, 0xbf80" : "=v"(k.cl));
  asm volatile("v_mov_b32 %0, 0xbf800000" : "=v"(k.ch));
  return k;
}
// The whole split in one asm statement with the non-destructive VOP3P v_dot2_f32_bf16 (the
// builtin selects the accumulating v_dot2c_f32_bf16, so each residual of a value that stays
// live -- the weights -- costs a v_mov first).  Wait states, all inside the string: a DOT
// result is read by another VALU instruction only >= 4 instructions later (the gfx950 rule is
// 3); the residual dots read the previous level's residual as their accumulator (SrcC); the
// string ends with s_nop 1 for the MFMAs that read hi / mid / lo as operands.
__device__ inline void split3(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo, SplitK K) {
  uint32_t h0, h1, h2, h3, m0, m1, m2, m3, o0, o1, o2, o3;
  float r0, r1, r2, r3, r4, r5, r6, r7;
  asm volatile(
      "v_cvt_pk_bf16_f32 %0, %20, %21\n\t"
      "v_cvt_pk_bf16_f32 %1, %22, %23\n\t"
      "v_cvt_pk_bf16_f32 %2, %24, %25\n\t"
      "v_cvt_pk_bf16_f32 %3, %26, %27\n\t"
      "v_dot2_f32_bf16 %12, %0, %28, %20\n\t"
      "v_dot2_f32_bf16 %13, %0, %29, %21\n\t"
      "v_dot2_f32_bf16 %14, %1, %28, %22\n\t"
      "v_dot2_f32_bf16 %15, %1, %29, %23\n\t"
      "v_dot2_f32_bf16 %16, %2, %28, %24\n\t"
      "v_dot2_f32_bf16 %17, %2, %29, %25\n\t"
      "v_dot2_f32_bf16 %18, %3, %28, %26\n\t"
      "v_dot2_f32_bf16 %19, %3, %29, %27\n\t"
      "v_cvt_pk_bf16_f32 %4, %12, %13\n\t"
      "v_cvt_pk_bf16_f32 %5, %14, %15\n\t"
      "v_cvt_pk_bf16_f32 %6, %16, %17\n\t"
      "v_dot2_f32_bf16 %12, %4, %28, %12\n\t"
      "v_dot2_f32_bf16 %13, %4, %29, %13\n\t"
      "v_cvt_pk_bf16_f32 %7, %18, %19\n\t"
      "v_dot2_f32_bf16 %14, %5, %28, %14\n\t"
      "v_dot2_f32_bf16 %15, %5, %29, %15\n\t"
      "v_dot2_f32_bf16 %16, %6, %28, %16\n\t"
      "v_dot2_f32_bf16 %17, %6, %29, %17\n\t"
      "v_dot2_f32_bf16 %18, %7, %28, %18\n\t"
      "v_dot2_f32_bf16 %19, %7, %29, %19\n\t"
      "v_cvt_pk_bf16_f32 %8, %12, %13\n\t"
      "v_cvt_pk_bf16_f32 %9, %14, %15\n\t"
      "v_cvt_pk_bf16_f32 %10, %16, %17\n\t"
      "s_nop 0\n\t"
      "v_cvt_pk_bf16_f32 %11, %18, %19\n\t"
      "s_nop 1"
      : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(m3),
        "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3), "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3),
        "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
        "v"(K.cl), "v"(K.ch));
  hi = __builtin_bit_cast(bf16x8, make_uint4(h0, h1, h2, h3));
  mid = __builtin_bit_cast(bf16x8, make_uint4(m0, m1, m2, m3));
  lo = __builtin_bit_cast(bf16x8, make_uint4(o0, o1, o2, o3));
}

// 8 bf16 of a transposed operand: two ds_read_b64_tr_b16 (rows lo .. lo + 3, hi .. hi + 3 of
// a 16-bit image in LDS; see T10 in cdna_hip_programming.md).  The whole wave must be active.
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4v;
__device__ inline bf16x8 tr_pair(const char* lo, const char* hi) {
  const short4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)lo);
  const short4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)hi);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ inline floatx4 mfma3(bf16x8 a, bf16x8 bhi, bf16x8 bmid, bf16x8 blo) {
  floatx4 z = {};
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, blo, z, 0, 0, 0);
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bmid, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bhi, z, 0, 0, 0);
}
__device__ inline floatx4 mfma3t(bf16x8 ahi, bf16x8 amid, bf16x8 alo, bf16x8 b) {
  floatx4 z = {};
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, b, z, 0, 0, 0);
  z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(amid, b, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, b, z, 0, 0, 0);
}

// The backward of one sample slot j of the sample-major layout (lane (g, c) holds samples
// 4g + j (j < 4) and 16 + 4g + j - 4 (j >= 4), hidden 16w + c), with the loss gradients
// x0..x2 of that sample taken from lane j of the lane's own row by DPP row_newbcast, fused
// into the FMAs (the loss lanes are laid out so that lane j of row g holds exactly that
// sample, see `ls` in k_chain3):
//   g2_k += h * x_k  (k = 0..2),   dh = fma(x2, W2_2, fma(x0, W2_0, x1 * W2_1))
// the same operations in the same order as the round-3 chain (which read the x_k back from
// an LDS copy of dL/dz2 and compiled (x0 W2_0 + x1 W2_1) + x2 W2_2 to exactly those fmas).  The compiler does not fuse a DPP
// move into v_fmac_f32, hence asm.  Hazard: a DPP source read >= 2 wait states after the
// VALU write of that register; the x_k are written before slot 0's statement, which starts
// with s_nop 1 (slot j + 1 reads slot j's g2 sums, so slot 0's statement comes first).  Not
// volatile: a volatile statement bounds the scheduler's regions, and the DPP chains of the
// totals (tot32) then lose the instructions that hide their hazards.
#define NFSP_BWD_DPP(L, NOP, OPG, CG)                                                       \
  asm(NOP                                                                                 \
               OPG " %0, %4, %7 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"            \
               OPG " %1, %5, %7 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"            \
               OPG " %2, %6, %7 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"            \
               "v_mul_f32_dpp %3, %5, %9 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"  \
               "v_fmac_f32_dpp %3, %4, %8 row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t" \
               "v_fmac_f32_dpp %3, %6, %10 row_newbcast:" #L " row_mask:0xf bank_mask:0xf"     \
               : CG(g0), CG(g1), CG(g2), "=&v"(dh)                                             \
               : "v"(x0), "v"(x1), "v"(x2), "v"(h), "v"(W0), "v"(W1), "v"(W2))
// slot 0 starts the g2 sums (a product, no accumulator register to zero)
template <int L>
__device__ inline float bwd_dpp(float& g0, float& g1, float& g2, float x0, float x1, float x2, float h,
                                float W0, float W1, float W2) {
  float dh;
  if constexpr (L == 0) NFSP_BWD_DPP(0, "s_nop 1\n\t", "v_mul_f32_dpp", "=&v");
  else if constexpr (L == 1) NFSP_BWD_DPP(1, "", "v_fmac_f32_dpp", "+v");
  else if constexpr (L == 2) NFSP_BWD_DPP(2, "", "v_fmac_f32_dpp", "+v");
  else if constexpr (L == 3) NFSP_BWD_DPP(3, "", "v_fmac_f32_dpp", "+v");
  else if constexpr (L == 4) NFSP_BWD_DPP(4, "", "v_fmac_f32_dpp", "+v");
  else if constexpr (L == 5) NFSP_BWD_DPP(5, "", "v_fmac_f32_dpp", "+v");
  else if constexpr (L == 6) NFSP_BWD_DPP(6, "", "v_fmac_f32_dpp", "+v");
  else NFSP_BWD_DPP(7, "", "v_fmac_f32_dpp", "+v");
  return dh;
}
#undef NFSP_BWD_DPP

// RELU: 0 = the AR net (softmax, categorical cross-entropy), 1 = the BR net (ReLU Q head,
// Huber), 2 = a BR net with a linear Q head (NFSP_EXT_LINEAR_Q, Huber), 3 = linear head with
// mean squared error (NFSP_EXT_MSE_Q).
// TABLE: the workgroups' jobs come from the device table C.jobs (engine groups); else from
// the kernel arguments (C.job, one engine) -- a separate instantiation, so the one-engine
// chain's code is not touched by the group's
template <int RELU, int LOSS, int TABLE = 0>
__global__ void __launch_bounds__(256) k_chain3(ChainArgs C) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Chain3Smem& sm = *reinterpret_cast<Chain3Smem*>(smem_raw);
  const ChainJob J = TABLE ? C.jobs[blockIdx.x] : C.job[blockIdx.x];
#include "chain3_body.inc"
}

// One job's chain as a device function (k_br_persist, learner.hip): the same body
template <int RELU, int LOSS, int TABLE>
__device__ __forceinline__ void chain3_run(const ChainArgs& C, const ChainJob J, char* smem_raw) {
  Chain3Smem& sm = *reinterpret_cast<Chain3Smem*>(smem_raw);
#include "chain3_body.inc"
}


// The chains' dynamic-LDS attribute (CHAIN_LDS), set once per device and kernel pair
// (`mask`: one bit per device, kept by the caller's translation unit).
inline int set_chain_lds(std::atomic<uint64_t>& mask, const void* f0, const void* f1, const void* f2,
                         const void* f3) {
  int dev = 0;
  NFSP_HIP(hipGetDevice(&dev));
  const uint64_t bit = 1ull << (dev & 63);
  if (mask.load(std::memory_order_acquire) & bit) return NFSP_OK;
  for (const void* f : {f0, f1, f2, f3})
    NFSP_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN_LDS));
  mask.fetch_or(bit, std::memory_order_acq_rel);
  return NFSP_OK;
}

// Launch k_chain3<RELU, loss_log, C.jobs != null> on `s` with `blocks` workgroups of C.lds
// (else CHAIN_LDS) bytes of LDS, after setting the LDS attribute of the four instantiations
// once per device.
template <int RELU>
int launch_chain(const ChainArgs& C, int blocks, bool loss_log, hipStream_t s, std::atomic<uint64_t>& attr) {
  const int rc = set_chain_lds(attr, (const void*)k_chain3<RELU, 0, 0>, (const void*)k_chain3<RELU, 1, 0>,
                               (const void*)k_chain3<RELU, 0, 1>, (const void*)k_chain3<RELU, 1, 1>);
  if (rc != NFSP_OK) return rc;
  const int lds = C.lds > 0 ? C.lds : CHAIN_LDS;
  if (lds < (int)sizeof(Chain3Smem) || lds > CHAIN_LDS) return nfsp::fail(NFSP_EINVAL, "chain LDS size");
  if (C.jobs) {
    if (loss_log) k_chain3<RELU, 1, 1><<<blocks, 256, lds, s>>>(C);
    else k_chain3<RELU, 0, 1><<<blocks, 256, lds, s>>>(C);
  } else {
    if (loss_log) k_chain3<RELU, 1, 0><<<blocks, 256, lds, s>>>(C);
    else k_chain3<RELU, 0, 0><<<blocks, 256, lds, s>>>(C);
  }
  NFSP_LAUNCHED("k_chain3");
  return NFSP_OK;
}

// AR chain launcher (chain_ar.hip): k_chain3<0, loss_log, *> on `s`, `blocks` workgroups.
int launch_chain_ar(const ChainArgs& C, int blocks, bool loss_log, hipStream_t s);
// BR chain with a linear Q head (NFSP_EXT_LINEAR_Q; chain_brlin.hip): k_chain3<2, loss_log>.
int launch_chain_br_linear(const ChainArgs& C, int blocks, bool loss_log, bool mse, hipStream_t s);

}  // namespace chain
}  // namespace nfsp

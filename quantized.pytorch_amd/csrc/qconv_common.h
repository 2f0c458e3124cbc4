// Definitions shared by the int8 contraction kernels (qconv.hip: 32x32x32 MFMA tiles,
// qconv16.hip: 16x16x64 MFMA tiles with LDS-staged input bands): launch parameters, the
// epilogue kinds, code stores and the LDS staging of the per-channel epilogue data.
#pragma once
#include <algorithm>

#include "qnn_internal.h"

namespace qnn {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int LDS_MAX = 160 * 1024;  // gfx950: LDS per CU

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

constexpr int MAX_TAPS = 64;
constexpr int MAX_CLASSES = 32;
constexpr int MAX_MASK = 1024;
constexpr int KPAD_ALIGN = 128;  // packed weight rows are multiples of 128 bytes (any BK divides)
constexpr int NUM_CU = 256;

enum { TAP_ONE = 0, TAP_TWO = 1, TAP_LDS = 2 };

struct Params {
  qnn_conv_desc d;
  qnn_epilogue e;
  int M;         // n*ho*wo
  int taps;      // kh*kw
  int lgcpt;     // log2(cp/16): 16-byte chunks per tap
  int kw_magic;  // ceil(2^16 / kw): t / kw == (t * kw_magic) >> 16 for t < 64
  int ct;        // C-tile columns, ceil(cout / 32)
  int stagger;   // 8-wave blocks: waves 4-7 refill after computing (QNN_CONV_STAGGER=0 disables)
  int epi_off;   // LDS byte offset of the epilogue data (stage_epi)
  int epi_early; // 1: staged by LDS-DMA at kernel start (lands during the main loop), 0: after it
  int scr_off;   // LDS byte offset of the NCHW transpose scratch (used after the main loop)
};

struct CodeDst {
  int8_t* ptr;
  int cp, pad, hp, wp;
};

__device__ __forceinline__ void store_codes(const CodeDst& t, int n, int ho, int wo, int ch, bool ok, v4i v) {
  if (ok && ch < t.cp)
    *reinterpret_cast<v4i*>(t.ptr + (((int64_t)n * t.hp + ho + t.pad) * t.wp + wo + t.pad) * t.cp + ch) = v;
}

// Epilogue kinds (one kernel instantiation each, so a kernel carries only its path):
//   EK_NCHW   mode 0: the drop-in fp32 NCHW output of QConv2d / QLinear
//   EK_LUT    conv -> RangeBN -> ReLU -> one consumer's codes via the per-channel table
//   EK_BNCODE conv -> RangeBN input codes only (stem before the code-domain max-pool)
//   EK_GEN    any other fused chain: [RangeBN] [+ residual] [ReLU] -> fp32 / codes x2
enum { EK_NCHW = 0, EK_LUT = 1, EK_BNCODE = 2, EK_GEN = 3 };

static inline int epi_kind(const qnn_epilogue& e) {
  if (e.mode == 0) return EK_NCHW;
  if (e.lut) return EK_LUT;
  if (e.out_bncode && !e.out_f32 && !e.out_code0 && !e.out_code1) return EK_BNCODE;
  return EK_GEN;
}

// Byte offset of lane `lane`'s 16 bytes of the 32x32 sub-tile (pixel tile mt, channel tile
// ctb) of a byte C-tile code map (include/qnn.h, qnn_res_link): lane-linear 1 KiB blocks.
__device__ __forceinline__ int64_t btile_off(int mt, int ctb, int ct, int lane) {
  return (((int64_t)mt * ct + ctb) * 64 + lane) * 16;
}

// Epilogue data in LDS at p.epi_off (f32 unless noted):
//   [0,BM) sxsw  [BM,2BM) sxbw  [2BM,3BM) bias  [3BM..7BM) bn mean/sq/wq/bq
//   [7BM, (7+nclass)BM) border table [cls][BM]  then (EK_LUT) int8 LUT [BM][256], or
//   (EK_GEN, residual code chain) [nres][mean/sq/wq/bq][BM] of the chain links
// moved by LDS-DMA (4 bytes per lane for the vectors and the table, 16 for the LUT), one
// job per wave-instruction, so the whole staging is ~8 DMA per wave and one round trip.
// Channels past cout read channel cout-1 (their outputs are never stored).
template <class C, int EK>
__device__ __forceinline__ void stage_epi(const Params& p, const int8_t* x, int8_t* dst, int c0, int wave, int lane) {
  constexpr int BM = C::BM, W = C::W, CH = BM / 64;  // 64-float chunks per vector
  const qnn_epilogue& e = p.e;
  const int cmax = p.d.cout - 1;
  const int nvec = (EK != EK_NCHW && e.bn_mean) ? 7 : 3;
  const int nf = (nvec + e.nclass + (EK == EK_GEN ? 4 * e.nres : 0)) * CH;
  for (int jb = wave; jb < nf; jb += W) {
    const int v = jb / CH, k = jb - v * CH;
    const int arr = v < nvec ? v : 7 + (v - nvec);
    int c = c0 + 64 * k + lane;
    c = c < cmax ? c : cmax;
    const float* src;
    switch (arr) {
      case 0: src = e.sxsw; break;
      case 1: src = e.sxbw; break;
      case 2:  // no bias: zeros from the input's 128-byte zero page
        if (!e.bias) {
          src = reinterpret_cast<const float*>(x + p.d.zero_off);
          c = lane & 31;
        } else {
          src = e.bias;
        }
        break;
      case 3: src = e.bn_mean; break;
      case 4: src = e.bn_sq; break;
      case 5: src = e.bn_wq; break;
      case 6: src = e.bn_bq; break;
      default:
        if (arr - 7 < e.nclass) {
          src = e.table + (int64_t)(arr - 7) * p.d.cout;
        } else {  // chain link l, vector k (mean, sq, wq, bq)
          const int lk = arr - 7 - e.nclass, l = lk >> 2, k = lk & 3;
          const qnn_res_link& r = e.res[l];
          src = k == 0 ? r.mean : k == 1 ? r.sq : k == 2 ? r.wq : r.bq;
        }
        break;
    }
    __builtin_amdgcn_global_load_lds((const void*)(src + c), (lds_ptr_t)(dst + 4 * (arr * BM + 64 * k)), 4, 0, 0);
  }
  if constexpr (EK == EK_LUT) {
    int8_t* lut = dst + 4 * (7 + e.nclass) * BM;
    for (int jl = wave; jl < BM / 4; jl += W) {
      int c = c0 + 4 * jl + (lane >> 4);
      c = c < cmax ? c : cmax;
      __builtin_amdgcn_global_load_lds((const void*)(e.lut + (int64_t)c * 256 + 16 * (lane & 15)),
                                       (lds_ptr_t)(lut + 1024 * jl), 16, 0, 0);
    }
  }
}

// Launch resources of one configuration (qnn_conv_occupancy): when a launch function is given
// an Occ it fills it and returns without launching.
struct Occ {
  int blocks_per_cu;  // co-resident blocks per CU at the launch's LDS (hipOccupancy...)
  int lds;            // dynamic LDS bytes per block
  int grid;           // blocks launched
};

// qconv16.hip's configurations (ids NCFG.. of qnn_conv_plan): count, tile, availability, cost, launch
int q16_count();
void q16_tile(int k, int* bm, int* bn);
bool q16_ok(int k, const Params& p);
double q16_cost(int k, const Params& p);
int q16_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s);
// qconv_rb.hip's resident-band configurations (ids after qconv16.hip's)
int rb_count();
void rb_tile(int k, int* bm, int* bn);
bool rb_ok(int k, const Params& p);
double rb_cost(int k, const Params& p);
int64_t rb_blocks(int k, const Params& p);
int rb_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr);
// qconv_direct.hip's short-K configurations (ids after the resident-band ones, through rb_*)
int direct_count();
void direct_tile(int k, int* bm, int* bn);
bool direct_ok(int k, const Params& p);
double direct_cost(int k, const Params& p);
int64_t direct_blocks(int k, const Params& p);
int direct_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr);

// qconv_rb.hip's streamed resident-band configurations (the last ids, after the extra ring tiles)
int rs_count();
void rs_tile(int k, int* bm, int* bn);
bool rs_ok(int k, const Params& p);
double rs_cost(int k, const Params& p);
int64_t rs_blocks(int k, const Params& p);
int rs_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr);

// qconv_rbp.hip's two-team resident-band configurations (ids after the direct ones)
int rbp_count();
void rbp_tile(int k, int* bm, int* bn);
bool rbp_ok(int k, const Params& p);
double rbp_cost(int k, const Params& p);
int64_t rbp_blocks(int k, const Params& p);
int rbp_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr);

// qconv_direct.hip's classifier-head configuration (the last id)
bool dhead_ok(const Params& p);
int64_t dhead_blocks(const Params& p);
int dhead_launch(const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr);

// qconv_direct.hip's table-epilogue configurations (ids after the two-team ones)
int dtab_count();
void dtab_tile(int k, int* bm, int* bn);
bool dtab_ok(int k, const Params& p);
double dtab_cost(int k, const Params& p);
int64_t dtab_blocks(int k, const Params& p);
int dtab_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr);

// qconv_pb.hip's persistent-band configurations (ids after the classifier head)
int pb_count();
void pb_tile(int k, int* bm, int* bn);
bool pb_ok(int k, const Params& p);
double pb_cost(int k, const Params& p);
int64_t pb_blocks(int k, const Params& p);
// qnn_qconv2d_fwd_nchw_f32: the drop-in's fp32 NCHW input and its quantizer (the persistent-band
// kernel quantizes it into its band buffers instead of reading a code tensor)
struct F32In {
  const float* x;
  int c, h, w, pad;
  float neg_min, scale, qmax;
};
int pb_launch(int k, const int8_t* x, const int8_t* w, const Params& p, hipStream_t s, Occ* occ = nullptr,
              const F32In* fin = nullptr);

// stem_pool.hip: the space-to-depth stem conv fused with RangeBN's input codes and
// MaxPool2d(3, 2, 1) (qnn_qconv2d_maxpool_fwd)
int stem_pool_launch(const int8_t* x, const int8_t* w, const Params& p, int pool_ho, int pool_wo, uint8_t* out_code,
                     const int8_t* lut0, const qnn_code_out& c0, const int8_t* lut1, const qnn_code_out& c1,
                     hipStream_t s);

}  // namespace qnn

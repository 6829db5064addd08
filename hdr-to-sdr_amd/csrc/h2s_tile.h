// h2s_tile.h — the tile kernel k_tile (the specialised fast path of the fused
// tone-map kernel), its instance table and a per-DBG dispatcher.  Included by
// h2s_fast.hip (product instances) and h2s_fast_dbg*.hip (debug instances),
// so the instances compile as separate translation units.
//
// Same chain as k_generic (h2s_kernels.hip) and oracle/h2s_oracle.c, restated
// for throughput on gfx950:
//  * one template instance per (transfer, operator, desat): the 8 steps a wave
//    runs per tile are straight-line code the compiler can interleave;
//  * chroma upsampling on integer-valued floats (exact), the 1/4, 1/8 and
//    depth-normalisation scales folded into the Y'CbCr->R'G'B' constants;
//  * the 3D-LUT lattice pre-multiplied into output Y'CbCr code space
//    (RGB->Y'CbCr is linear and the lattice lies in [0,1], so the swscale
//    clip is a no-op and blend-then-convert == convert-then-blend); the
//    tetrahedral blend then yields quantiser inputs directly;
//  * lattice gathers are buffer loads (32-bit offsets, one SGPR base);
//  * eq's table sits in LDS.
// Geometry (k_tile): a block of 256 threads walks 8 consecutive 64 x 32 luma
// tiles, prefetching tile i+1 into registers while tile i computes.  A tile
// (Y, and U/V with their 1-row halo) is staged into LDS with coalesced
// 16-byte loads; then, in 8 steps, each wave processes one dense 8 x 8 pixel
// sub-block with one pixel per lane (lanes 4q..4q+3 = one 2x2 quad).  Dense
// sub-blocks keep the 64 lanes of every lattice gather on few cache lines;
// chroma is reduced per quad with DPP quad permutes and all outputs leave
// through LDS as 16-byte coalesced stores.  Measured balance (DESIGN.md
// §4.1): VALU ~70 % busy, LDS ~47 %, vector-memory return ~35 %.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "h2s_device.h"

// Round-4 VALU trims of the step (on by default, each
// switchable for A/B builds, scripts/build_variants.sh):
//  H2S_TAGSEL    tetrahedron from axis-tagged fractions + a 3-entry LDS
//                offset table, one-key uniformity test (9 + 6 half-rate ops -> 6)
//  (EXPCLAMP)    lut3d's [0, N-1] clamp as v_exp_f32's output clamp
//  H2S_EQMAGIC   eq index by a 2^23 add and a 16-bit shift (full-rate ops)
// The PQ table's first segment (E' < 1/128, below ~0.0015 nits), where the
// EOTF ~ (E - E0)^6.28 and no cubic holds 1e-3 relative, is staged as the
// cubic FLT_MAX t: exactly 0 at E = 0 (black, common in real content), and
// above DARK_MARK for every E in (0, 1/128).  The pixel's luma sum (or an
// explicit probe) carries such a channel to one wave-wide test; the rare
// waves that meet it re-run S1 and S2 with those channels exact.  No
// per-channel range test in the common path.
#ifndef H2S_TAGSEL
#define H2S_TAGSEL 1
#endif
#ifndef H2S_EQMAGIC
#define H2S_EQMAGIC 1
#endif
// Stage markers for the per-stage slot table (scripts/isa_stages.py): in a
// marked build (-DH2S_ISA_MARKS, ISA listing only, never linked) each is an
// assembler comment ";@@name" that opens stage `name` in the listing, with a
// scheduling barrier so that no instruction crosses it; the product build
// defines them away
#ifdef H2S_ISA_MARKS
#define H2S_MARK(name)                  \
  do {                                  \
    __builtin_amdgcn_sched_barrier(0);  \
    asm volatile(";@@" name);           \
    __builtin_amdgcn_sched_barrier(0);  \
  } while (0)
// the same, with three values pinned to the marker (read and rewritten by
// it), so that the IR passes cannot sink their computation past it
#define H2S_MARKV(name, a, b, c)                                  \
  do {                                                            \
    __builtin_amdgcn_sched_barrier(0);                            \
    asm volatile(";@@" name : "+v"(a), "+v"(b), "+v"(c));         \
    __builtin_amdgcn_sched_barrier(0);                            \
  } while (0)
#else
#define H2S_MARK(name)
#define H2S_MARKV(name, a, b, c)
#endif

namespace h2s {

typedef float f3 __attribute__((ext_vector_type(3)));

typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

// a global pointer held in a VGPR pair (address space 1: the loads through it
// are global_load, counted in vmcnt only -- a flat load would also count in
// lgkmcnt, so every LDS wait would wait for it too)
typedef __attribute__((address_space(1))) const unsigned gu32;
__device__ __forceinline__ gu32* in_vgpr64(const unsigned* x) {
  gu32* y;
  asm volatile("v_mov_b64 %0, %1" : "=v"(y) : "s"((gu32*)x));
  return y;
}

// streaming frame I/O: non-temporal so the pixels do not evict LUT lines
__device__ __forceinline__ uint2 nt_ld2(const uint8_t* p) {
  const u2v v = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p));
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint4 nt_ld4(const uint8_t* p) {
  const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_st2(uint2 w, uint8_t* p) {
  __builtin_nontemporal_store(u2v{w.x, w.y}, reinterpret_cast<u2v*>(p));
}
__device__ __forceinline__ void nt_st4(uint4 w, uint8_t* p) {
  __builtin_nontemporal_store(u4v{w.x, w.y, w.z, w.w}, reinterpret_cast<u4v*>(p));
}


__device__ __forceinline__ long long fxcd_remap(long long b, long long nb) {
  const long long xcd = b & 7, idx = b >> 3, per = nb >> 3, rem = nb & 7;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

// exact zimg st_2084_eotf x 2^log2_scale (S1: 10000/npl for PQ input; used
// above the table's range and in its first segment)
__device__ __forceinline__ float pq_exact_s(float e, float log2_scale) {
  const float xp = fexp2(flog2(fmaxf(e, 0.0f)) * (1.0f / PQ_M2));
  const float num = fmaxf(xp - PQ_C1, 0.0f);
  const float den = fmaxf(PQ_C2 - PQ_C3 * xp, 1.17549435e-38f);  // zimg: max(.., FLT_MIN)
  return fexp2(flog2(num * frcp(den)) * (1.0f / PQ_M1) + log2_scale);
}
__device__ __forceinline__ float pq_exact(const FastParams& F, float e) { return pq_exact_s(e, F.log2_lin_scale); }


// Zero-segment form used by k_tile: the LDS table holds a zero segment at
// index 0 and segment i of pq_tab at i+1, and the caller passes
// u = E*PQ_SEG + 1 (the +1 is folded into the staged luma).  v_cvt_u32_f32
// saturates negatives to 0, so E < 0 reads the zero segment (EOTF = 0) with no
// clamp; at and past PQZ_LIM the value is garbage and the caller takes the
// exact path.  The byte offset is formed with a 16-bit shift (full rate; bits
// 31:16 are written as zero on gfx950, and the index fits 12 bits).
__device__ __forceinline__ float pq_z(const float4* tab, float u) {
  unsigned off;
  asm("v_cvt_u32_f32 %0, %1\n\tv_lshlrev_b16 %0, 4, %0" : "=v"(off) : "v"(u));
  const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tab) + off);
  const float t = __builtin_amdgcn_fractf(u);
  return fmaf(fmaf(fmaf(c.x, t, c.y), t, c.z), t, c.w);
}
// staged E (table-segment units, +1) at and above which pq_z is invalid
constexpr float PQZ_LIM = PQ_EMAX * (float)PQ_SEG + 1.0f;

// legitimate table values stay below ~1e10 (E < 1.875); the marked first
// segment gives >= FLT_MAX 2^-23 = 4e31 for any E > 0
constexpr float DARK_MARK = 1e30f;

// the EOTF-table read with its first segment (staged u in (1, 2)) evaluated
// exactly instead: the dark re-run of a wave (px_chain).  Only the lanes in
// that segment take the exact form (a divergent branch inside the rare re-run)
__device__ __forceinline__ float pq_z_dark(const float4* tab, float u, float log2_scale) {
  float v = pq_z(tab, u);
  if (u > 1.0f && u < 2.0f) v = pq_exact_s((u - 1.0f) * (1.0f / (float)PQ_SEG), log2_scale);
  return v;
}

// ST 2084 inverse EOTF of y = luminance / 10000 >= 0 from the LDS table
// (build_pqi_table): the segment is the float's exponent and top three
// mantissa bits, t the remaining 20 mantissa bits as [0, 1/8); the bit
// pattern is clamped (as a signed integer) to the table's octaves 2^-64 ..
// 2^14, where one pattern below the first octave reads entry 0, the constant
// PQ(0) = c1^m2: y <= 0 (black, or an LMS row of a saturated colour) exactly
// as the oracle's max(y, 0), and y below 2^-64 (1e-15 nits, within 3e-7 of
// PQ(0)).  The IPT form caps its input at 1e6 npl, inside the top octave.
// The near-black octaves matter: an LMS row of a dark pixel on synthetic
// content reaches 1e-13, and clamping at 2^-40 (PQ 1.4e-5 instead of down to
// 7.3e-7) put 0.5 % errors on stage-2 values of 1e-5.  Eight segments per
// octave, not four (round 5): the LMS encode error the decode amplifies (x
// ~11-45 through the EOTF's slope) drops from ~1e-6 to the float32 floor
// (scripts/c3_table_flips.py: the rgba8 download flips this table alone
// causes drop 7x); the 10 KB table puts the libplacebo instances above 32 KB
// of LDS, i.e. at 4 blocks per CU.  Round 6: 8 VALU instructions (integer
// med3, bfe, shift-add, and-or, add, 3 FMA) instead of 13 -- the clamp on the
// pattern replaces the segment clamp and the y <= 0 select
__device__ __forceinline__ float pqi(const float4* tab, float y) {
  constexpr int S0 = (127 + PQI_OCT0) << 3;                  // absolute segment of 2^-64
  constexpr int LO = (S0 - 1) << 20;                         // reads entry 0
  constexpr int HI = ((S0 + PQI_NSEG) << 20) - 1;            // the top segment's last pattern
  const int bc = min(max(__builtin_bit_cast(int, y), LO), HI);   // (v_med3_i32)
  unsigned sa;
  asm("v_bfe_u32 %0, %1, 20, 11" : "=v"(sa) : "v"(bc));      // absolute segment (sign bit is 0)
  const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tab) + ((sa - (unsigned)(S0 - 1)) << 4));
  const float t = __builtin_bit_cast(float, ((unsigned)bc & 0xFFFFFu) | 0x3F800000u) - 1.0f;
  return fmaf(fmaf(fmaf(c.x, t, c.y), t, c.z), t, c.w);
}

// S1 transfer to linear (units of npl), specialised
// returns true (wave-uniform) when some lane of the wave took the exact PQ
// path: linear values may then be huge or infinite, and the tone curve must
// use its overflow-safe form
// NOEX: the caller knows no E reaches the table's end (a tile of legal codes,
// see k_tile): no ballot, no exact path, so a step has no branch
// DARK: the table's first segment exactly (pq_z_dark) instead of the NaN
template <int TRC, int ESC = 1, bool NOEX = false, bool DARK = false>
__device__ __forceinline__ bool to_linear(const FastParams& F, const float4* pq_lds, float er, float eg, float eb,
                                          float& r, float& g, float& b) {
  if (TRC == 0) {
    // E arrives as E*PQ_SEG + 1 (pq_z)
    static_assert(TRC != 0 || ESC == PQ_SEG, "PQ staging is in table-segment units");
    if (DARK) {
      r = pq_z_dark(pq_lds, er, F.log2_lin_scale), g = pq_z_dark(pq_lds, eg, F.log2_lin_scale);
      b = pq_z_dark(pq_lds, eb, F.log2_lin_scale);
    } else {   // a channel in the table's first segment is marked here (px_chain's dark re-run)
      r = pq_z(pq_lds, er), g = pq_z(pq_lds, eg), b = pq_z(pq_lds, eb);
    }
    constexpr float EI = 1.0f / (float)PQ_SEG;
    // NOEX (the fast body): the tile's codes keep every E inside the table
    // (tflag): no exact path above it, no ballot for it
    if (NOEX) return false;
    const float emax = __builtin_fmaxf(__builtin_fmaxf(er, eg), eb);
    const bool high = __builtin_amdgcn_ballot_w64(emax >= PQZ_LIM) != 0;   // rare: extreme out-of-gamut codes
    if (high) {
      r = er >= PQZ_LIM ? pq_exact(F, (er - 1.0f) * EI) : r;
      g = eg >= PQZ_LIM ? pq_exact(F, (eg - 1.0f) * EI) : g;
      b = eb >= PQZ_LIM ? pq_exact(F, (eb - 1.0f) * EI) : b;
    }
    return high;
  } else {
    // zimg arib_b67_inverse_oetf, branch-free; then the OOTF (gamma 1.2)
    auto inv = [](float e) -> float {
      const float x = fmaxf(e, 0.0f);
      const float lo = (x * x) * (1.0f / 3.0f);
      const float hi = (fexp2((x - HLG_C) * (1.4426950408889634f / HLG_A)) + HLG_B) * (1.0f / 12.0f);
      return x <= 0.5f ? lo : hi;
    };
    if (ESC == PQ_SEG) {
      // the CPU chain's instances: the inverse OETF from the same LDS cubic
      // table layout as the PQ EOTF (build_hlg_table; E staged as
      // E*PQ_SEG + 1), the direct form past the table
      r = pq_z(pq_lds, er), g = pq_z(pq_lds, eg), b = pq_z(pq_lds, eb);
      const float emax = __builtin_fmaxf(__builtin_fmaxf(er, eg), eb);
      constexpr float EI = 1.0f / (float)PQ_SEG;
      if (!NOEX && __builtin_amdgcn_ballot_w64(emax >= PQZ_LIM)) {
        r = er >= PQZ_LIM ? inv((er - 1.0f) * EI) : r;
        g = eg >= PQZ_LIM ? inv((eg - 1.0f) * EI) : g;
        b = eb >= PQZ_LIM ? inv((eb - 1.0f) * EI) : b;
      }
    } else {
      r = inv(er), g = inv(eg), b = inv(eb);
    }
    const float ys = 0.2627f * r + 0.6780f * g + 0.0593f * b;
    const float w = fexp2(flog2(ys) * 0.2f + F.log2_lin_scale);  // ys == 0 -> 0
    r *= w, g *= w, b *= w;
    return false;  // HLG is bounded (E <= 2.2 -> a few 1e4)
  }
}

// S2 vf_tonemap, specialised.  DESAT: 0 off, 1 weighted luma (F.lr/lg/lb),
// 2 the RGB-coefficient luma r+g+b (vf_tonemap's table entry for the linear
// RGB frame zscale hands it; the default).
//
// Bounded form (every lane's linear values from the PQ table or HLG, so
// sig <= ~6e8 and den*sig cannot overflow): the desaturation and the gain
// fold into out = c*A + B with A = (1-ob)*k, B = L*ob*k, since
// max(c*(1-ob) + L*ob) = max(c)*(1-ob) + L*ob for 0 <= ob <= 1; the curve
// uses one reciprocal.  Safe form (the wave met the exact PQ path): the
// statement order of vf_tonemap, two reciprocals.
//
// BT.2390 on PQ input (TRC 0, bounded form): the EETF's first step encodes
// sig = max(R,G,B) back to PQ, and PQ(EOTF(max E)) = max E, so e1 is the
// input's own max code value (emax_s = max E * PQ_SEG + 1, clamped below at
// the code of sig = 1e-6); the final decode reads the EOTF table in LDS.
// libplacebo branch with h2s_lp_tone IPT (F.lp_ipt): the curve acts on the
// intensity of IPT-PQ instead (three LMS rows encoded through the PQ-encode
// table, L'M'S' += I' - I decoded through the EOTF table), as the oracle's
// tone_ipt.
// DARK: the dark re-run (px_chain): every EOTF-table read takes its first
// segment exactly (pq_z_dark) instead of the mark staged there.  luma: the
// desaturation's luma (DESAT instances), the CPU chain's free dark probe
template <int TRC, int TM, int DESAT, int LP, bool DARK = false>
__device__ __forceinline__ void tone(const FastParams& F, const CurveConsts& C, const float4* pq_lds,
                                     const float4* pqi_lds, float& r, float& g, float& b, bool safe, float emax_s,
                                     float hable_kb, float& luma_out) {
  auto pz = [&](float u) { return DARK ? pq_z_dark(pq_lds, u, F.log2_pq_scale) : pq_z(pq_lds, u); };
  if (LP && TM >= 4 && TM <= 6) {
    // libplacebo's reinhard / hable / mobius (scaling PL_HDR_NORM: 1 = the
    // target white; oracle lp_norm_curve), on the IPT intensity or as the
    // max(R,G,B) gain; the frame's constants come from its curve record
    auto curve = [&](float x) -> float {
      x = __builtin_amdgcn_fmed3f(x, 0.0f, C.n_peak);
      if (TM == 4) return C.n_rein_scale * x / (x + C.n_rein_off);
      if (TM == 5) return hable(x) * C.n_hable_inv;
      return x <= C.n_mob_j ? x : C.n_mob_scale * (x + C.n_mob_a) / (x + C.n_mob_b);
    };
    const float R = fminf(r, 1e6f), G = fminf(g, 1e6f), B = fminf(b, 1e6f);
    if (F.lp_ipt) {
      const float q0 = pqi(pqi_lds, F.ipt_r2l[0] * R + F.ipt_r2l[1] * G + F.ipt_r2l[2] * B);
      const float q1 = pqi(pqi_lds, F.ipt_r2l[3] * R + F.ipt_r2l[4] * G + F.ipt_r2l[5] * B);
      const float q2 = pqi(pqi_lds, F.ipt_r2l[6] * R + F.ipt_r2l[7] * G + F.ipt_r2l[8] * B);
      const float I = 0.4f * q0 + 0.4f * q1 + 0.2f * q2;
      const float x = pz(fmaf(I, (float)PQ_SEG, 1.0f)) * F.tw_fold;     // NORM
      luma_out = x;   // (marked for a dark I: the curve's clamp below would drop it; px_chain probes it)
      const float I2 = pqi(pqi_lds, curve(x) * F.tw_1e4);
      const float du = fmaf(I2 - I, (float)PQ_SEG, 1.0f);
      auto lz = [&](float q) { return pz(__builtin_amdgcn_fmed3f(fmaf(q, (float)PQ_SEG, du), 1.0f, PQZ_LIM - 0.01f)); };
      const float l0 = lz(q0), l1 = lz(q1), l2 = lz(q2);
      r = F.ipt_l2r[0] * l0 + F.ipt_l2r[1] * l1 + F.ipt_l2r[2] * l2;
      g = F.ipt_l2r[3] * l0 + F.ipt_l2r[4] * l1 + F.ipt_l2r[5] * l2;
      b = F.ipt_l2r[6] * l0 + F.ipt_l2r[7] * l1 + F.ipt_l2r[8] * l2;
    } else {
      const float sig = fmaxf(__builtin_fmaxf(__builtin_fmaxf(R, G), B), 1e-6f);
      const float k = curve(sig * F.n_nw) / sig;
      r = R * k, g = G * k, b = B * k;
    }
    return;
  }
  if (TM == 7 || TM == 8) {  // BT.2390 / spline (PQ-domain curves, no desat)
    // PQ input: the curve straight into pq_z's table coordinate u = e4*PQ_SEG
    // + 1 (the output scale and offset are folded into the polynomial
    // coefficients on the host, resolve_fast)
    auto curve_u = [&](float e1) -> float {
      float u;
      if (TM == 7) {   // BT.2390 Hermite knee as one cubic in t, Horner form
        const float e1n = __builtin_amdgcn_fmed3f(fmaf(e1, C.b_e1a, C.b_e1b), 0.0f, 1.0f);
        const float t = fmaf(e1n, C.b_ta, C.b_tb);
        const float uk = fmaf(fmaf(fmaf(C.b_c3, t, C.b_c2), t, C.b_c1), t, C.b_c0);
        u = e1n > C.b_thr ? uk : fmaf(e1n, C.b_lr, C.b_lc);
        if (C.b_minlum > 0.0f) {   // libplacebo black-point adaptation (block-uniform branch)
          const float om = fmaf(u, C.b_bk_a, C.b_bk_b);          // 1 - e2
          float pw;
          if (C.b_bp == 4.0f) {
            const float o2 = om * om;
            pw = o2 * o2;
          } else {
            pw = fexp2(C.b_bp * flog2(fmaxf(om, 0.0f)));
          }
          const float ub = fmaf(pw, C.b_bk_c, fmaf(u, C.b_gain, C.b_bk_d));
          u = om > 0.0f ? ub : u;
        }
      } else {         // spline: cubic shoulder / quadratic toe around the knee
        const float x = __builtin_amdgcn_fmed3f(e1, C.sp_srcmin, C.sp_srcmax) - C.sp_kin;
        const float uq = fmaf(fmaf(fmaf(C.sp_qa_u, x, C.sp_qb_u), x, C.sp_qc_u), x, C.sp_k_u);
        const float up = fmaf(fmaf(C.sp_pa_u, x, C.sp_pb_u), x, C.sp_k_u);
        u = __builtin_amdgcn_fmed3f(x > 0.0f ? uq : up, C.sp_umin, C.sp_umax);
      }
      return u;
    };
    // HLG input: the curve's PQ output e4
    auto curve_e4 = [&](float e1) -> float {
      if (TM == 7) {
        const float e1n = fmaxf(fminf((e1 - C.b_srcmin) * C.b_inv_range, 1.0f), 0.0f);
        const float t = (e1n - C.b_ks) * C.b_inv_1mks;
        const float t2 = t * t, t3 = t2 * t;
        const float p = (2.0f * t3 - 3.0f * t2 + 1.0f) * C.b_ks + (t3 - 2.0f * t2 + t) * (1.0f - C.b_ks) +
                        (-2.0f * t3 + 3.0f * t2) * C.b_maxlum;
        const float e2 = bt2390_black(C.b_minlum, C.b_bp, C.b_gain, (C.b_ks < 1.0f && e1n > C.b_ks) ? p : e1n);
        return fmaxf(e2 * C.b_range + C.b_srcmin, 0.0f);   // <= source max <= 1
      }
      return spline_pq(C, e1);                              // within [PQ(0), PQ(npl)]
    };
    auto eotf_exact = [](float e) -> float {   // normalised (1 = 10000 nits), e in [0, ~1.1]
      const float xp = fexp2(flog2(fmaxf(e, 0.0f)) * (1.0f / PQ_M2));
      return fexp2(flog2(fmaxf(xp - PQ_C1, 0.0f) * frcp(PQ_C2 - PQ_C3 * xp)) * (1.0f / PQ_M1));
    };
    auto pq_enc = [](float y) -> float {       // y = luminance / 10000
      const float ym = fexp2(flog2(fmaxf(y, 0.0f)) * PQ_M1);
      return fexp2(flog2((PQ_C1 + PQ_C2 * ym) * frcp(1.0f + PQ_C3 * ym)) * PQ_M2);
    };
    if (LP && F.lp_ipt) {   // (LP instances only: they stage both tables)
      // libplacebo branch, h2s_lp_tone IPT (oracle tone_ipt): the curve on
      // the intensity of IPT-PQ with P and T kept, i.e. L'M'S' += I' - I;
      // encode and decode through the LDS tables (launch-uniform branch; the
      // EOTF table is staged for HLG input too)
      H2S_MARK("S2a RGB->LMS, PQ encode x3");
      const float R = fminf(r, 1e6f), G = fminf(g, 1e6f), B = fminf(b, 1e6f);
      const float q0 = pqi(pqi_lds, F.ipt_r2l[0] * R + F.ipt_r2l[1] * G + F.ipt_r2l[2] * B);
      const float q1 = pqi(pqi_lds, F.ipt_r2l[3] * R + F.ipt_r2l[4] * G + F.ipt_r2l[5] * B);
      const float q2 = pqi(pqi_lds, F.ipt_r2l[6] * R + F.ipt_r2l[7] * G + F.ipt_r2l[8] * B);
      H2S_MARK("S2b I, curve");
      const float I = 0.4f * q0 + 0.4f * q1 + 0.2f * q2;
      const float du = curve_u(I) - I * (float)PQ_SEG;   // (I' - I) PQ_SEG + 1
      H2S_MARK("S2c EOTF x3, LMS->RGB");
      auto lz = [&](float q) { return pz(__builtin_amdgcn_fmed3f(fmaf(q, (float)PQ_SEG, du), 1.0f, PQZ_LIM - 0.01f)); };
      const float l0 = lz(q0), l1 = lz(q1), l2 = lz(q2);
      r = F.ipt_l2r[0] * l0 + F.ipt_l2r[1] * l1 + F.ipt_l2r[2] * l2;
      g = F.ipt_l2r[3] * l0 + F.ipt_l2r[4] * l1 + F.ipt_l2r[5] * l2;
      b = F.ipt_l2r[6] * l0 + F.ipt_l2r[7] * l1 + F.ipt_l2r[8] * l2;
      return;
    }
    const float sig = fmaxf(__builtin_fmaxf(__builtin_fmaxf(r, g), b), 1e-6f);
    float e1;
    if (TRC == 0 && !safe) {
      e1 = fmaxf(fmaf(emax_s, 1.0f / (float)PQ_SEG, -1.0f / (float)PQ_SEG), F.b_e1min);
    } else {  // exact PQ encode: HLG input, or the wave met the exact EOTF path
      e1 = pq_enc(sig * F.npl_1e4);
    }
    // EOTF(e4) * 10000/target white (TRC 0: the table is npl-scaled)
    const float s2 = TRC == 0 ? pz(curve_u(e1)) * F.tw_fold : eotf_exact(curve_e4(e1)) * F.e4_npl;
    const float k = safe ? s2 / sig : s2 * frcp(sig);   // IEEE division on the exact path (see below)
    r *= k, g *= k, b *= k;
    return;
  }
  if (safe) {
    // the wave met the exact PQ path: linear values up to ~1e38 or inf.
    // vf_tonemap's statement order with IEEE division, as the generic kernel
    // (tonemap_px): v_rcp_f32 flushes the (denormal) reciprocal of anything
    // above 8.5e37 to zero, which Hable's num/den reaches at sig ~ 2.7e19
    if (DESAT) {
      const float luma = DESAT == 2 ? (r + g) + b : F.lr * r + F.lg * g + F.lb * b;
      luma_out = luma;
      const float ob = fmaxf(luma - F.desat, 1e-6f) / fmaxf(luma, 1e-6f);
      r = r * (1.0f - ob) + luma * ob;
      g = g * (1.0f - ob) + luma * ob;
      b = b * (1.0f - ob) + luma * ob;
    }
    const float sig = fmaxf(__builtin_fmaxf(__builtin_fmaxf(r, g), b), 1e-6f);
    float t;
    if (TM == 4) {  // REINHARD
      t = sig / (sig + F.rein_p) * F.rein_k;
    } else if (TM == 5) {  // HABLE
      t = hable(sig) * F.hable_peak_inv;
    } else {  // MOBIUS: identity below j
      t = sig <= F.mob_j ? sig : F.mob_k * (sig + F.mob_a) / (sig + F.mob_b);
    }
    const float k = t / sig;
    r *= k, g *= k, b *= k;
    return;
  }
  float sig, A = 1.0f, B = 0.0f;
  if (DESAT) {
    const float luma = DESAT == 2 ? (r + g) + b : F.lr * r + F.lg * g + F.lb * b;
    luma_out = luma;
    const float ob = fmaxf(luma - F.desat, 1e-6f) * frcp(fmaxf(luma, 1e-6f));
    A = 1.0f - ob, B = luma * ob;
    sig = fmaxf(fmaf(__builtin_fmaxf(__builtin_fmaxf(r, g), b), A, B), 1e-6f);
  } else {
    sig = fmaxf(__builtin_fmaxf(__builtin_fmaxf(r, g), b), 1e-6f);
  }
  float k;
  if (TM == 4) {
    k = F.rein_k * frcp(sig + F.rein_p);
  } else if (TM == 5) {
    // hable(x) = N/D - e/f with 15 N - D = x (2.1 x + 0.25) (the constant
    // terms cancel: d*e*15 = d*f), so hable(x)/x = (0.14 x + 1/60) / D:
    // one reciprocal, no cancellation, and sig drops out of the gain
    const float den = fmaf(sig, fmaf(sig, 0.15f, 0.50f), 0.06f);
    k = fmaf(sig, F.hable_ka, hable_kb) * frcp(den);   // (kb in a VGPR: one scalar operand per VOP3)
  } else {
    const float m = F.mob_k * (sig + F.mob_a) * frcp((sig + F.mob_b) * sig);
    k = sig <= F.mob_j ? 1.0f : m;
  }
  if (DESAT) {
    A *= k, B *= k;
    r = fmaf(r, A, B), g = fmaf(g, A, B), b = fmaf(b, A, B);
  } else {
    r *= k, g *= k, b *= k;
  }
}

// S3 + S4 coordinates: s = clamp((N-1) * x^(1/2.4)), as lattice units
// NaN -> 0 (lut3d sanitizef), +inf -> top of the lattice
__device__ __forceinline__ float lut_s(const FastParams& F, float x) {
  return fminf(fmaxf(fexp2(flog2(x) * (1.0f / 2.4f) + F.log2_nm1), 0.0f), F.s_max);
}


// hot constants the kernels keep in VGPRs for their whole run (in_vgpr)
struct StepK {
  float a_rv, a_gv, a_gu, a_bu;   // chroma terms of E, x ESC
  float stride_g, stride_b;       // lattice byte strides (as floats)
  int og, ob, ocr, ocg, ocb;      // corner byte offsets
  float log2_nm1, x_max;
  float hable_kb;                 // F.hable_kb (Hable instances)
  int c111;                       // the far corner's byte offset
  float nm1;                      // N - 1
  const int* offtab;              // LDS: byte offset of the +1 corner along r, g, b at bytes 0, 4, 8
  float lp_k2, lp_hi, lp_cy;      // LP: the encode's clamp bounds lp_k2, 255 + lp_k2; lp_cy + ydq
  float lp_k1;                    // LP: the encode's exponent offset (a VGPR: it meets a literal)
};

// S1 + S2 of one pixel (px_chain, lp_front): staged luma ybs (Y*ys + y_off,
// +1 on PQ), x8-upsampled centred chroma U, V -> the tone-mapped linear
// R, G, B, with the dark re-run below.  dput: the debug planes' writer (DBG)
template <int TRC, int TM, int DESAT, int LP, int DBG, bool NOEX, class DPut>
__device__ __forceinline__ void lin_tone(const FastParams& F, const CurveConsts& cv, const float4* pq_lds,
                                         const float4* pqi_lds, const StepK& K, float ybs, float U, float V,
                                         const DPut& dput, float& r, float& gg, float& bl) {
  // E in table-segment units for the table forms: the PQ EOTF, and the HLG
  // inverse OETF on the CPU chain (the libplacebo branch keeps direct HLG)
  constexpr int ESC = TRC == 0 || !LP ? PQ_SEG : 1;
  H2S_MARK("S1a E");
  const float er = fmaf(V, K.a_rv, ybs);
  const float eg = fmaf(V, K.a_gv, fmaf(U, K.a_gu, ybs));
  const float eb = fmaf(U, K.a_bu, ybs);
  H2S_MARK("S1b EOTF");
  const bool safe = to_linear<TRC, ESC, NOEX>(F, pq_lds, er, eg, eb, r, gg, bl);
  H2S_MARKV("S2 tone", r, gg, bl);
  if (DBG == 1) {   // the stage-1 planes with the first segment exact, as the dark re-run below gives them
    float r1, g1, b1;
    to_linear<TRC, ESC, NOEX, true>(F, pq_lds, er, eg, eb, r1, g1, b1);
    dput(r1, g1, b1);
  }
  const float emax_s = __builtin_fmaxf(__builtin_fmaxf(er, eg), eb);
  // S1's own marked channels are probed before the tone map wherever the
  // tone map can drop the mark: the libplacebo branch's IPT form caps its
  // input at 1e6 npl, and a max(R,G,B) gain without desaturation scales the
  // marked channel back to the curve's output (k = curve(sig) / sig)
  constexpr bool S1P = TRC == 0 && (LP || !(DESAT && TM <= 6));
  const float s1probe = S1P ? (r + gg) + bl : 0.0f;
  float luma = 0.0f;
  tone<TRC, TM, DESAT, LP>(F, cv, pq_lds, pqi_lds, r, gg, bl, safe, emax_s, K.hable_kb, luma);
  H2S_MARKV("S2z dark probe", r, gg, bl);
  // The EOTF table's first segment is marked wherever it is read (S1 on PQ
  // input; the libplacebo branch's IPT decode and curve reads): a value that
  // reached it is huge (> DARK_MARK) in S1's output or the tone map's.  The
  // CPU chain's desaturating instances see it in their luma for free, the
  // others sum the channels' magnitudes (and S1's, S1P); a wave that meets one re-runs S1 and S2
  // with that segment evaluated exactly (about 1 % of the bench content's
  // 8x8 steps)
  if constexpr (TRC == 0 || LP) {
    float probe;
    if constexpr (!LP && DESAT && TM <= 6) {
      probe = luma;
    } else {
      probe = (fabsf(r) + fabsf(gg)) + fabsf(bl);   // (the IPT rows mix signs: magnitudes do not cancel)
      if constexpr (S1P) probe += s1probe;
      if constexpr (LP && TM >= 4 && TM <= 6) probe += luma;   // the NORM curve's decoded intensity
    }
    if (__builtin_amdgcn_ballot_w64(!(probe <= DARK_MARK))) {   // (NaN / inf from a marked value too)
      H2S_MARK("rare: dark re-run");
      const bool safe2 = to_linear<TRC, ESC, NOEX, true>(F, pq_lds, er, eg, eb, r, gg, bl);
      tone<TRC, TM, DESAT, LP, true>(F, cv, pq_lds, pqi_lds, r, gg, bl, safe2, emax_s, K.hable_kb, luma);
    }
  }
}

// The libplacebo branch's rgba8 download and lut3d table read (S3, S4) of one
// pixel from its tone-mapped linear R, G, B: the BT.1886 encode against the
// target black, 255 x it rounded to the 8-bit rgba code (qoff: the range=tv
// and rounding / dither offsets, h2s_lp_range / _dither, less lp_k2 lp_qs_f:
// the encode's - lp_k2 is folded into the clamp's bounds K.lp_k2 / K.lp_hi;
// all offsets >= 0, so the conversion's truncation is the floor).
// Everything after the download -- lut3d's 8-bit coordinate (q / 255)
// (N-1), the tetrahedral blend in vf_lut3d's order, the truncation to 8 bits
// -- is a function of the three codes alone, so it is one read of the
// context's 2^24-entry table of lut3d's 8-bit outputs (k_build_lut8x: the
// generic kernel's own lut3d_8bit arithmetic, bit for bit), instead of a
// lattice cell, four gathers and the blend per pixel (round 6, VERDICT r05
// item 2).  Returns the table entry (R | G << 8 | B << 16) as loaded: the
// caller decides where to wait for it
__device__ __forceinline__ unsigned lp_table_read(const FastParams& F, const StepK& K, gu32* lut8v,
                                                  const unsigned* spread_lds, float r, float gg, float bl,
                                                  float qoff) {
  auto q8 = [&](float x) -> unsigned {
    const float e = fexp2(fmaf(flog2(__builtin_amdgcn_fmed3f(x, 0.0f, F.lp_xmax)), 1.0f / 2.4f, K.lp_k1));
    return (unsigned)fmaf(__builtin_amdgcn_fmed3f(e, K.lp_k2, K.lp_hi), F.lp_qs_f, qoff);
  };
  unsigned idx;
  const unsigned qr = q8(r), qg = q8(gg), qb = q8(bl);
  H2S_MARK("S4 lut3d table read");
  // the table's bit-interleaved (Morton) index: nearby colours share lines
  asm("v_lshl_or_b32 %0, %1, 1, %2" : "=v"(idx) : "v"(spread_lds[qb]), "v"(spread_lds[qg]));
  asm("v_lshl_or_b32 %0, %1, 1, %2" : "=v"(idx) : "v"(idx), "v"(spread_lds[qr]));
  // (a global load from a 64-bit VGPR base, one shift-add for the address:
  // the table's buffer descriptor took four SGPRs that the LP instances
  // spill, i.e. four lane reads per step)
  return lut8v[idx];
}

// BT.709 limited-range Y'CbCr at depth q straight from lut3d's 8-bit output
// codes (FastParams lp_ky / lp_kcb / lp_kcr: the rows x 1/255 x the depth
// scales, folded on the host): o = (luma code + 0.5, 56 q Cb, 56 q Cr)
__device__ __forceinline__ f3 lp_ycbcr(const FastParams& F, const StepK& K, float R8, float G8, float B8) {
  f3 o;
  o.x = fmaf(F.lp_ky[0], R8, fmaf(F.lp_ky[1], G8, fmaf(F.lp_ky[2], B8, K.lp_cy)));
  o.y = fmaf(F.lp_kcb[0], R8, fmaf(F.lp_kcb[1], G8, F.lp_kcb[2] * B8));
  o.z = fmaf(F.lp_kcr[0], R8, fmaf(F.lp_kcr[1], G8, F.lp_kcr[2] * B8));
  return o;
}

// One pixel through S1..S7 (both tile kernels): staged luma ybs (Y*ys +
// y_off, +1 on PQ), x8-upsampled centred chroma U, V -> the eq'd luma code at
// the output depth (returned) and the pixel's two chroma quantiser
// contributions (oyv, ozv) for the 2x2 sum.  di: this pixel's index in the
// debug planes (DBG > 0, frame 0), else -1.  (The libplacebo branch's
// product steps run lin_tone / lp_table_read / lp_ycbcr software-pipelined
// instead: k_tile's steps.)
template <int TRC, int TM, int DESAT, int LP, int DBG, bool NOEX = false>
__device__ __forceinline__ unsigned px_chain(const FastParams& F, const CurveConsts& cv, const float4* pq_lds,
                                             const float4* pqi_lds, const uint16_t* eq_lds, gu32* lut8v, const unsigned* spread_lds,
                                             __amdgpu_buffer_rsrc_t lut, const StepK K, float ybs, float U, float V,
                                             long long di, float& oyv, float& ozv, float qoff, float ydq) {
  constexpr bool EQM = H2S_EQMAGIC && !LP;   // see the eq lookup at the end
  const long long dpl = (long long)F.dbg_w * F.H;
  auto dput = [&](float a, float b_, float c) {
    if (di >= 0) F.dbg[di] = a, F.dbg[dpl + di] = b_, F.dbg[2 * dpl + di] = c;
  };
  float r, gg, bl;
  lin_tone<TRC, TM, DESAT, LP, DBG, NOEX>(F, cv, pq_lds, pqi_lds, K, ybs, U, V, dput, r, gg, bl);
  H2S_MARKV("S3 encode", r, gg, bl);
  if (DBG == 2) dput(r, gg, bl);
  f3 o;
  if (LP && F.lut_off) {
    // LUT off: libplacebo's BT.2020 -> BT.709 matrix on the linear
    // values, the BT.1886 encode clipped to [0, 1] (no rgba rounding: the
    // branch downloads nv12), then Y'CbCr at depth q as below
    // (255-scaled, into the same folded Y'CbCr rows as the 8-bit codes below)
    auto enc = [&](float x) -> float {
      const float e = fexp2(fmaf(flog2(__builtin_amdgcn_fmed3f(x, 0.0f, F.lp_xmax)), 1.0f / 2.4f, F.lp_k1)) - F.lp_k2;
      return __builtin_amdgcn_fmed3f(e, 0.0f, 255.0f);
    };
    const float R = enc(F.m709[0] * r + F.m709[1] * gg + F.m709[2] * bl);
    const float G = enc(F.m709[3] * r + F.m709[4] * gg + F.m709[5] * bl);
    const float B = enc(F.m709[6] * r + F.m709[7] * gg + F.m709[8] * bl);
    if (DBG == 3 || DBG == 4) dput(R * F.inv255, G * F.inv255, B * F.inv255);
    o.x = fmaf(F.lp_ky[0], R, fmaf(F.lp_ky[1], G, fmaf(F.lp_ky[2], B, K.lp_cy)));
    o.y = fmaf(F.lp_kcb[0], R, fmaf(F.lp_kcb[1], G, F.lp_kcb[2] * B));
    o.z = fmaf(F.lp_kcr[0], R, fmaf(F.lp_kcr[1], G, F.lp_kcr[2] * B));
  } else if constexpr (LP) {
    if (DBG == 3) {
      auto ev = [&](float x) {
        const float e = fexp2(fmaf(flog2(__builtin_amdgcn_fmed3f(x, 0.0f, F.lp_xmax)), 1.0f / 2.4f, F.lp_k1)) - F.lp_k2;
        return __builtin_amdgcn_fmed3f(e, 0.0f, 255.0f) * F.inv255;
      };
      dput(ev(r), ev(gg), ev(bl));
    }
    const unsigned v = lp_table_read(F, K, lut8v, spread_lds, r, gg, bl, qoff);
    const float R8 = (float)(v & 255u), G8 = (float)((v >> 8) & 255u), B8 = (float)((v >> 16) & 255u);   // (v_cvt_f32_ubyte0..2)
    H2S_MARK("S5 Y'CbCr");
    if (DBG == 4) dput(R8 * F.inv255, G8 * F.inv255, B8 * F.inv255);
    o = lp_ycbcr(F, K, R8, G8, B8);
  } else {
    // lattice cell origins (cr, cg, cb) and fractions (dr, dg, db) per channel
    float cr, cg, cb, dr, dg, db;
    {
      float sr, sg, sb;
      // S3+S4: s = (N-1) x^(1/2.4) with x clamped to [0, K.x_max] (NaN -> 0), so
      // s < N-1 and the lattice cell index never needs a clamp
      // lut3d's clamp to [0, N-1] (NaN -> 0) as the exp's output clamp:
      // x^(1/2.4) clamped to [0, 1] (v_exp_f32 ... clamp; a NaN from the log
      // of a negative or NaN x clamps to 0), then N - 1 times that.  s may
      // reach N-1 exactly: its corners past the lattice edge get weight 0
      // (zero fraction), and the lattice allocation is padded for them
      sr = __builtin_amdgcn_fmed3f(fexp2(flog2(r) * (1.0f / 2.4f)), 0.0f, 1.0f) * K.nm1;
      sg = __builtin_amdgcn_fmed3f(fexp2(flog2(gg) * (1.0f / 2.4f)), 0.0f, 1.0f) * K.nm1;
      sb = __builtin_amdgcn_fmed3f(fexp2(flog2(bl) * (1.0f / 2.4f)), 0.0f, 1.0f) * K.nm1;
      // s is a product when N-1 is not a power of two (N-1 times the clamped
      // power): without this barrier the compiler contracts the cell origin
      // s - fract(s) below into fma(N-1, x, -fract(s)), which carries the
      // product's rounding error, so the origin is no longer an integer and a
      // byte offset truncates to a misaligned record (N = 177: 45 of 3072
      // samples of a uniform frame)
      asm("" : "+v"(sr), "+v"(sg), "+v"(sb));
      H2S_MARKV("S4a cell, fractions", sr, sg, sb);
      dr = __builtin_amdgcn_fractf(sr), dg = __builtin_amdgcn_fractf(sg), db = __builtin_amdgcn_fractf(sb);
      cr = sr - dr, cg = sg - dg, cb = sb - db;
    }
    H2S_MARKV("S4b tetrahedron select", dr, dg, db);
    const int base = (int)fmaf(cb, K.stride_b, fmaf(cg, K.stride_g, cr * 12.0f));
    // H2S_TAGSEL (the CPU chain): tetrahedron by sorting axis-tagged
    // fractions: the 4 low mantissa bits of each fraction carry its axis a
    // (bits 3:2 and 1:0 both = a; r 0, g 1, b 2; a change of <= 2^-19
    // relative in the weights), so max3 / min3 / med3 of the bit patterns
    // (non-negative floats order as integers) give the sorted fractions and
    // the axes of the largest and smallest; the corner offsets come from a
    // 3-entry LDS table (om = +1 along the max axis, ocn = the far corner less
    // the min axis), not from compares and selects (9 half-rate VALU ops ->
    // 3).  (Not for the libplacebo branch's 8-bit coordinates, whose exact
    // ties between fractions the tags would break: that branch reads its
    // table above.)
    constexpr bool TAG = H2S_TAGSEL;
    int om, ocn;
    float dmax, dmin, dmid;
    unsigned umin = 0, amax = 0;
    if constexpr (TAG) {
      const unsigned ur = __builtin_bit_cast(unsigned, dr) & ~15u;
      const unsigned ug = (__builtin_bit_cast(unsigned, dg) & ~15u) | 5u;
      const unsigned ub = (__builtin_bit_cast(unsigned, db) & ~15u) | 10u;
      unsigned umax, umid;
      asm("v_max3_u32 %0, %1, %2, %3" : "=v"(umax) : "v"(ur), "v"(ug), "v"(ub));
      asm("v_min3_u32 %0, %1, %2, %3" : "=v"(umin) : "v"(ur), "v"(ug), "v"(ub));
      asm("v_med3_u32 %0, %1, %2, %3" : "=v"(umid) : "v"(ur), "v"(ug), "v"(ub));
      amax = umax & 12u;
      const unsigned amin = umin & 12u;
      om = *reinterpret_cast<const int*>(reinterpret_cast<const char*>(K.offtab) + amax);
      ocn = K.c111 - *reinterpret_cast<const int*>(reinterpret_cast<const char*>(K.offtab) + amin);
      dmax = __builtin_bit_cast(float, umax), dmin = __builtin_bit_cast(float, umin), dmid = __builtin_bit_cast(float, umid);
    } else {
      const bool rg = dr > dg, gb = dg > db, rb = dr > db;
      om = rg ? (rb ? 12 : K.ob) : (gb ? K.og : K.ob);
      ocn = rg ? (gb ? K.ocb : K.ocg) : (rb ? K.ocb : K.ocr);
      dmax = __builtin_fmaxf(__builtin_fmaxf(dr, dg), db);
      dmin = __builtin_fminf(__builtin_fminf(dr, dg), db);
      dmid = __builtin_amdgcn_fmed3f(dr, dg, db);
    }
    H2S_MARKV("S4c weights, uniformity, gathers, blend", dmax, dmid, dmin);
    const float w0 = 1.0f - dmax, w1 = dmax - dmid, w2 = dmid - dmin, w3 = dmin;
    auto blend = [&](const f3 c0, const f3 c1, const f3 c2, const f3 c3) {
      f3 r = w0 * c0 + w1 * c1 + w2 * c2 + w3 * c3;
      // the luma quantiser's ordered-dither offset (ydq = d - 0.5, 0 without
      // dither: the record's +0.5 rounds) as the blend's first term (FMA for MUL)
      r.x = fmaf(w3, c3.x, fmaf(w2, c2.x, fmaf(w1, c1.x, fmaf(w0, c0.x, ydq))));
      return r;
    };
    // when every lane of the step is in one cell and one tetrahedron, its
    // four records come through the scalar cache and the step issues no
    // vector-memory gather (bit-identical; C2 -1.8 % smooth, -5 % on the
    // website frame: profiles/r03/ablations/sgather_*.log)
    bool step_uniform;
    int b0, m0, n0;
    if constexpr (TAG) {
      // one key per lane: cell (base) and tetrahedron (the max and min axes)
      unsigned tkey, key;
      asm("v_and_or_b32 %0, %1, 3, %2" : "=v"(tkey) : "v"(umin), "v"(amax));
      asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(key) : "v"(base), "v"(tkey));
      const unsigned key0 = __builtin_amdgcn_readfirstlane(key);
      step_uniform = __builtin_amdgcn_ballot_w64(key != key0) == 0;
      b0 = 0, m0 = 0, n0 = 0;
      if (step_uniform) {
        b0 = (int)(key0 >> 4);
        m0 = __builtin_amdgcn_readfirstlane(om), n0 = __builtin_amdgcn_readfirstlane(ocn);
      }
    } else {
      b0 = __builtin_amdgcn_readfirstlane(base), m0 = __builtin_amdgcn_readfirstlane(om),
      n0 = __builtin_amdgcn_readfirstlane(ocn);
      step_uniform = __builtin_amdgcn_ballot_w64(base != b0 || om != m0 || ocn != n0) == 0;
    }
    if (step_uniform) {
      typedef __attribute__((address_space(4))) const float cfl;
      cfl* L = (cfl*)F.lut_yuv;
      auto sl = [&](int off) {
        const int i = off >> 2;
        return f3{L[i], L[i + 1], L[i + 2]};
      };
      o = blend(sl(b0), sl(b0 + m0), sl(b0 + n0), sl(b0 + F.c111));
    } else {
      o = blend(__builtin_amdgcn_raw_buffer_load_b96(lut, base, 0, 0), __builtin_amdgcn_raw_buffer_load_b96(lut, base + om, 0, 0),
                __builtin_amdgcn_raw_buffer_load_b96(lut, base + ocn, 0, 0),
                __builtin_amdgcn_raw_buffer_load_b96(lut, base, F.c111, 0));
    }
    if (DBG == 3) dput((cr + dr) * F.inv_nm1, (cg + dg) * F.inv_nm1, (cb + db) * F.inv_nm1);   // = s exactly
    if (DBG == 4) {  // same cell / corners / weights on the RGB lattice (12-byte record -> float4 index)
      const float4 q0 = F.dbg_lut[base / 12], q1 = F.dbg_lut[(base + om) / 12], q2 = F.dbg_lut[(base + ocn) / 12],
                   q3 = F.dbg_lut[(base + F.c111) / 12];
      dput(w0 * q0.x + w1 * q1.x + w2 * q2.x + w3 * q3.x, w0 * q0.y + w1 * q1.y + w2 * q2.y + w3 * q3.y,
           w0 * q0.z + w1 * q1.z + w2 * q2.z + w3 * q3.z);
    }
  }
  H2S_MARKV("S7 eq", o.x, o.y, o.z);
  if (DBG == 5) dput(o.x - (EQM ? 0.0f : 0.5f) - ydq, 4.0f * o.y, 4.0f * o.z);
  oyv = o.y, ozv = o.z;
  if constexpr (EQM) {
    // o.x = the luma quantiser input less 0.5 (the lattice records carry no
    // +0.5): adding 2^23 rounds it to the nearest integer in the mantissa's
    // low bits, and a 16-bit shift turns that into the table's byte offset
    // (two full-rate ops instead of a conversion and a 32-bit shift-add; an
    // exact .5 tie rounds to even instead of up: continuous blends of the
    // CPU chain, not the libplacebo branch's 8-bit-derived values)
    const unsigned qb = __builtin_bit_cast(unsigned, o.x + 8388608.0f);
    unsigned off;
    asm("v_lshlrev_b16 %0, 1, %1" : "=v"(off) : "v"(qb));
    return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(eq_lds) + off);
  } else {
    return eq_lds[(int)o.x];
  }
}

constexpr int CBW = 32, CBH = 16;  // chroma tile
#ifndef H2S_YST
#define H2S_YST 72
#endif
// LDS row stride (floats) of the staged luma tile and of the horizontally
// upsampled chroma rows.  72 on the CPU chain's instances: a step's 8 rows x 8
// columns then start 8 banks apart and cover all 64 banks (68 overlapped
// 2-way: 34 % -> 20 % of LDS-active cycles in bank conflicts, time unchanged;
// profiles/r04/ablations/lds_stride.txt).  68 on the libplacebo instances,
// whose PQ-encode table and native-depth eq table leave no room: +1.1 KB there
// drops them from 5 blocks per CU to 4 (C3 +9 %).  Round 5: their 8-segment
// PQ-encode table puts them at 4 blocks per CU anyway; 72 measured the same
// as 68 there (0.939 / 0.936 ms, profiles/r05/lp_variants.log), 68 kept for
// the LDS (the 12-bit output's 8 KB eq table)
#ifndef H2S_YST_LP
#define H2S_YST_LP 68
#endif
template <int LP>
constexpr int row_stride() { return LP ? H2S_YST_LP : H2S_YST; }
// buffer-op aux bits: non-temporal (streamed frame bytes).  Frame loads that
// bypass the L1 (sc1 nt, sc0 sc1 nt) or use workgroup scope (sc0 nt) time the
// same within 1 %: the streamed bytes do not evict the lattice lines the
// gathers wait on (profiles/r03/ablations/frame_load_cache_policy.log)
#ifndef H2S_NT_LOAD
#define H2S_NT_LOAD 2
#endif
#ifndef H2S_NT_STORE
#define H2S_NT_STORE 2
#endif
constexpr int NT = H2S_NT_LOAD, NTS = H2S_NT_STORE;   // cache-policy bits (ablation builds override)

__device__ __forceinline__ float quad_sum(float v) {
  // (v0 + v1) + (v2 + v3) over the 2x2 pixels of a quad, in all 4 lanes
  // (quad_perm [1,0,3,2] pairs horizontally, then [2,3,0,1] adds the rows):
  // the oracle's summation order, so the chroma sum is bit-identical.  (The
  // lane moves as ds_swizzle through the LDS crossbar with full-rate adds:
  // 2-3 % slower, the swizzle latency sits in every step's chain;
  // profiles/r03/ablations/quad_sum_swizzle_*.log)
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
}

__device__ __forceinline__ void unpack8(const uint4 a, float* o) {
  o[0] = (float)(a.x & 0xffff), o[1] = (float)(a.x >> 16), o[2] = (float)(a.y & 0xffff), o[3] = (float)(a.y >> 16);
  o[4] = (float)(a.z & 0xffff), o[5] = (float)(a.z >> 16), o[6] = (float)(a.w & 0xffff), o[7] = (float)(a.w >> 16);
}

// keep a wave-uniform constant in a VGPR (avoids per-use SGPR->VGPR moves
// forced by the one-scalar-operand limit of VOP3 on gfx950)
template <class T>
__device__ __forceinline__ T in_vgpr(T x) {
  T y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "s"(x));
  return y;
}

// bytes: the plane's extent, clamped to 2^31-1 on the host (FastParams in/out_bytes)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const uint8_t* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}

// one tile's global loads, held in registers between issue and the LDS commit
struct TileRegs {
  uint4 ya, ua;     // luma chunk; chroma chunk of plane pc (threads tc < 72)
  uint16_t uh;      // the chroma chunk's right-halo sample
};

struct TileGeo {
  int f, px0, py0, cx0, cy0;
};

// frame f's curve record: a constant-address-space load with a block-uniform
// index, so the compiler emits scalar (s_load) reads
__device__ __forceinline__ CurveConsts curve_of(const CurveConsts* frames, int f) {
  typedef __attribute__((address_space(4))) const float cfloat;
  constexpr int n = (int)(sizeof(CurveConsts) / sizeof(float));
  cfloat* src = (cfloat*)frames + __builtin_amdgcn_readfirstlane(f) * n;
  CurveConsts r;
  float* dst = reinterpret_cast<float*>(&r);
#pragma unroll
  for (int i = 0; i < n; i++) dst[i] = src[i];
  return r;
}

__device__ __forceinline__ TileGeo tile_geo(const FastParams& F, unsigned tile) {
  const unsigned bx = tile % F.nbx, bt = tile / F.nbx;
  TileGeo g;
  g.f = (int)(bt / F.nby);
  const int by = (int)(bt % F.nby);
  g.px0 = (int)bx * TBW, g.py0 = by * TBH, g.cx0 = (int)bx * CBW, g.cy0 = by * CBH;
  return g;
}

// the tile after g in walk order (x, then y, then frame): block-uniform
// scalar arithmetic, no division
__device__ __forceinline__ void tile_next(const FastParams& F, TileGeo& g) {
  g.px0 += TBW, g.cx0 += CBW;
  if (g.px0 >= F.W) {
    g.px0 = 0, g.cx0 = 0, g.py0 += TBH, g.cy0 += CBH;
    if (g.py0 >= (int)F.nby * TBH) g.py0 = 0, g.cy0 = 0, g.f++;
  }
}

// per-lane byte offsets of a tile's loads and stores relative to the tile's
// origin, fixed for the whole launch (the strides do not change): interior
// tiles then address with one scalar origin (soffset) and no per-lane
// arithmetic
struct LaneOfs {
  int y, u;        // loads: luma row yr, chunk yc; chroma row clr, chunk ccx of plane pc
  int sy, sc;      // stores: luma row / 8-sample chunk; chroma row of plane pl
};

__device__ __forceinline__ LaneOfs lane_ofs(const FastParams& F, int t) {
  LaneOfs L;
  L.y = (t >> 3) * (int)F.in_ls[0] + 16 * (t & 7);
  const int pc = (t >> 7) & 1, tc = t & 127;
  L.u = (tc >> 2) * (int)F.in_ls[1 + pc] + 16 * (tc & 3);
  const int sb = F.out8 ? 8 : 16;
  L.sy = (t >> 3) * (int)F.out_ls[0] + sb * (t & 7);
  const int pl = (t >> 6) & 1, rem = t & 63;
  L.sc = (rem >> 2) * (int)F.out_ls[1 + pl] + sb * (rem & 3);
  return L;
}

// issue (do not wait for) the loads of one tile: luma 64 x 32 (one 16-byte
// load per thread) and chroma rows cy0-1 .. cy0+16 (18 rows x 4 chunks of 8
// samples + 1 right-halo sample): plane U on threads 0..71, plane V on threads
// 128..199, so waves 0-1 and 2-3 share the chroma work and the plane (hence the
// buffer resource) is wave-uniform.  Tiles whose rows (and chroma
// halo) lie inside the frame take the lane offsets of LaneOfs plus a scalar
// origin; border tiles clamp per lane.  The chroma registers of threads >= 72
// are left undefined (never committed).
__device__ __forceinline__ TileRegs tile_load(const FastParams& F, const TileGeo& g, int t, const LaneOfs& L) {
  // Every thread issues exactly one load of each kind whatever the tile: the
  // offsets are chosen per case and the loads follow the merge; threads
  // without a chroma chunk read out of range, which returns 0 and fetches
  // nothing
  const __amdgpu_buffer_rsrc_t iy = plane_rsrc(F.in[0] + g.f * F.in_fp[0], F.in_bytes[0]);
  const int yr = t >> 3, yc = t & 7;
  TileRegs r;
  int vy, sy;
  if (g.py0 + TBH <= F.H) {   // block-uniform
    vy = L.y, sy = g.py0 * (int)F.in_ls[0] + 2 * g.px0;
  } else {
    vy = (g.py0 + yr < F.H ? g.py0 + yr : F.H - 1) * (int)F.in_ls[0] + 2 * (g.px0 + 8 * yc), sy = 0;
  }
  r.ya = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(iy, vy, sy, NT));
  const int pc = __builtin_amdgcn_readfirstlane(t >> 7), tc = t & 127;
  const __amdgpu_buffer_rsrc_t ic = plane_rsrc(F.in[1 + pc] + g.f * F.in_fp[1 + pc], F.in_bytes[1 + pc]);
  const int ls = (int)F.in_ls[1 + pc];
  int vc, vh, sc;
  if (g.cy0 >= 1 && g.cy0 + CBH + 1 <= F.ch && g.cx0 + CBW + 1 <= F.cw) {   // block-uniform
    vc = L.u, vh = L.u + 16, sc = (g.cy0 - 1) * ls + 2 * g.cx0;
  } else {
    const int clr = tc >> 2, ccx = tc & 3;
    const int row = chroma_edge_at(g.cy0 - 1 + clr, F.ch, F.chroma_edge);
    vc = row * ls + 2 * (g.cx0 + 8 * ccx);
    vh = row * ls + 2 * chroma_edge_at(g.cx0 + 8 * ccx + 8, F.cw, F.chroma_edge);
    sc = 0;
  }
  if (tc >= 72) vc = vh = 0x7FFFFFF0;
  r.ua = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ic, vc, sc, NT));
  r.uh = __builtin_amdgcn_raw_buffer_load_b16(ic, vh, sc, 0);
  return r;
}

// staging and store helpers of k_tile
// 8 luma samples -> Y*ys + y_off floats at (row, 8 col8)
// returns the largest staged value
template <int YST>
__device__ __forceinline__ float stage_luma(float* yin, uint4 a, int row, int col8, float ysc, float yoff) {
  float v[8];
  unpack8(a, v);
  float* d = yin + row * YST + 8 * col8;
  const float4 lo = make_float4(fmaf(v[0], ysc, yoff), fmaf(v[1], ysc, yoff), fmaf(v[2], ysc, yoff), fmaf(v[3], ysc, yoff));
  const float4 hi = make_float4(fmaf(v[4], ysc, yoff), fmaf(v[5], ysc, yoff), fmaf(v[6], ysc, yoff), fmaf(v[7], ysc, yoff));
  *reinterpret_cast<float4*>(d) = lo;
  *reinterpret_cast<float4*>(d + 4) = hi;
  return __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(lo.x, lo.y), __builtin_fmaxf(lo.z, lo.w)),
                         __builtin_fmaxf(__builtin_fmaxf(hi.x, hi.y), __builtin_fmaxf(hi.z, hi.w)));
}
// horizontal pass (left siting, x2 scale) on centred codes c = code - mid:
// h[2k] = 2 c[k], h[2k+1] = c[k] + c[k+1]; exact in float.  tt: chunk index
// (row tt >> 2, 8-sample chunk tt & 3) of the tile's 18 x 4 chroma chunks
// returns the largest |centred code|
template <int HST>
__device__ __forceinline__ float stage_chroma(float* plane, uint4 a, unsigned h, int tt, float cmid) {
  float v[9];
  unpack8(a, v);
  v[8] = (float)h;
#pragma unroll
  for (int k = 0; k < 9; k++) v[k] -= cmid;
  float m = fabsf(v[0]);
#pragma unroll
  for (int k = 1; k < 9; k++) m = __builtin_fmaxf(m, fabsf(v[k]));
  float* d = plane + (tt >> 2) * HST + 16 * (tt & 3);
#pragma unroll
  for (int k = 0; k < 4; k++)
    *reinterpret_cast<float4*>(d + 4 * k) =
        make_float4(v[2 * k] + v[2 * k], v[2 * k] + v[2 * k + 1], v[2 * k + 1] + v[2 * k + 1], v[2 * k + 1] + v[2 * k + 2]);
  return m;
}
// luma codes of tile row r, chunk c (8 pixels), packed for one 16-byte (u16)
// / 8-byte (u8: .xy) store
template <int YST>
__device__ __forceinline__ u4v read_luma(const FastParams& F, const float* yin, int r, int c) {
  const unsigned* src = reinterpret_cast<const unsigned*>(yin) + r * YST + 8 * c;
  const uint4 a = *reinterpret_cast<const uint4*>(src), b = *reinterpret_cast<const uint4*>(src + 4);
  if (F.out8)
    return u4v{a.x | (a.y << 8) | (a.z << 16) | (a.w << 24), b.x | (b.y << 8) | (b.z << 16) | (b.w << 24), 0u, 0u};
  return u4v{a.x | (a.y << 16), a.z | (a.w << 16), b.x | (b.y << 16), b.z | (b.w << 16)};
}
__device__ __forceinline__ void put_luma(const FastParams& F, const TileGeo& g, u4v v, int r, int vo, int so) {
  if (g.py0 + r >= F.H) return;
  const __amdgpu_buffer_rsrc_t oy_ = plane_rsrc(F.out[0] + g.f * F.out_fp[0], F.out_bytes[0]);
  so += g.py0 * (int)F.out_ls[0];
  if (F.out8)
    __builtin_amdgcn_raw_buffer_store_b64(u2v{v.x, v.y}, oy_, vo, so + g.px0, NTS);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, oy_, vo, so + 2 * g.px0, NTS);
}
// chroma plane pl, row r, chunk c (8 samples): ((c0 + c1) + (c2 + c3)) + bias,
// quantised once per sample, packed as read_luma
__device__ __forceinline__ u4v read_chroma(const FastParams& F, const float* csum, int pl, int r, int c) {
  const float4* src = reinterpret_cast<const float4*>(csum + pl * (CBH * CBW) + r * CBW + 8 * c);
  const float4 v0 = src[0], v1 = src[1];
  const float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  unsigned code[8];
  if (F.dither) {   // S6 ordered dither: sample (cx, cy) mod 8 = (k, r mod 8)
#pragma unroll
    for (int k = 0; k < 8; k++) code[k] = (unsigned)(int)(vv[k] + (F.c_bias - 0.5f + dither_off(k, r)));
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) code[k] = (unsigned)(int)(vv[k] + F.c_bias);
  }
  if (F.rep_rs == 31) {   // plain shift (block-uniform); else bit replication (h2s_expand)
#pragma unroll
    for (int k = 0; k < 8; k++) code[k] <<= F.shift_out;
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) code[k] = (code[k] << F.shift_out) | (code[k] >> F.rep_rs);
  }
  if (F.out8)
    return u4v{code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24),
               code[4] | (code[5] << 8) | (code[6] << 16) | (code[7] << 24), 0u, 0u};
  return u4v{code[0] | (code[1] << 16), code[2] | (code[3] << 16), code[4] | (code[5] << 16), code[6] | (code[7] << 16)};
}
__device__ __forceinline__ void put_chroma(const FastParams& F, const TileGeo& g, u4v v, int pl, int r, int vo) {
  if (g.cy0 + r >= F.ch) return;
  const __amdgpu_buffer_rsrc_t oc_ = plane_rsrc(F.out[1 + pl] + g.f * F.out_fp[1 + pl], F.out_bytes[1 + pl]);
  const int so = g.cy0 * (int)F.out_ls[1 + pl];
  if (F.out8)
    __builtin_amdgcn_raw_buffer_store_b64(u2v{v.x, v.y}, oc_, vo, so + g.cx0, NTS);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, oc_, vo, so + 2 * g.cx0, NTS);
}

// Each block walks F.tpb consecutive tiles (XCD-remapped, so neighbouring
// tiles and their lattice cells share one XCD's L2).  The loads of tile i+1
// are issued before tile i is computed, so after the first tile the block no
// longer waits on HBM latency.  Per tile: commit registers -> LDS, prefetch,
// barrier, 8 compute steps, barrier, store, barrier.  (A fifth wave doing all
// of the frame I/O, so that the compute waves' gathers never wait behind the
// prefetch in the shared vector-memory counter, measured 1.5x slower: its
// serial store + commit phase idles the four compute waves;
// profiles/r03/ablations/io_wave*.  Issuing the stores of tile i-1 and the
// loads of tile i+1 inside step 7, behind its gathers, measured 3-5 % slower:
// profiles/r03/ablations/late_io*.)
// DBG (debug instances only, never launched by h2s_process): 1..5 = also
// write that h2s_stage's three float planes for frame 0 to F.dbg (W x H each)
// from this kernel's own arithmetic — stage 4 blends the float4 RGB lattice
// F.dbg_lut with the same cell, corners and weights as the Y'CbCr lattice.
// LP = 1: the libplacebo branch (src/utils.py:444-460, BT.2390 / spline):
// BT.1886 encode against the target black, 8-bit rgba download, lut3d's 8-bit
// path on plain R'G'B' records (truncating output), BT.709 Y'CbCr at depth q
template <int TRC, int TM, int DESAT, int LP, int DBG = 0>
// 5 waves per SIMD = the LDS-bound occupancy (5 blocks of ~27.6 KB per CU;
// 3, 4 and 6 measured slower on the bench content, 6 by 4.5 % in round 3 at
// 80 VGPRs: profiles/r03/ablations/six_waves.log, blocks_per_cu.log): let
// the compiler use the VGPRs that allows
#ifndef H2S_TILE_WPE
#define H2S_TILE_WPE 5
#endif
// the libplacebo instances: the same 5 waves per SIMD for the register
// budget (96 VGPRs, 2-6 spilled); 4 (106 VGPRs, no spills) measured 8 %
// slower with the PQ-encode table's branch-free form (profiles/r05/lp_variants.log)
#ifndef H2S_TILE_WPE_LP
#define H2S_TILE_WPE_LP H2S_TILE_WPE
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LP ? H2S_TILE_WPE_LP : H2S_TILE_WPE))) void k_tile(
    const FastParams F) {
  constexpr int YST = row_stride<LP>(), HST = YST;
  __shared__ float yin[TBH * YST];             // luma samples x ys; output codes overwrite them in place
  __shared__ float hrow[2][(CBH + 2) * HST];   // chroma rows (halo incl.) upsampled x2 horizontally
  __shared__ float csum[2][CBH * CBW];         // per chroma sample: sum of its 2x2 pixel contributions
  __shared__ float4 pq_lds[PQ_NSEG + 1];       // [0] = zero segment (pq_z): PQ EOTF, or HLG inverse OETF (!LP)
  __shared__ float4 pqi_lds[LP ? PQI_NTAB : 1];                   // PQ encode (lp_tone IPT)
  extern __shared__ uint16_t eq_lds[];         // eq table, codes pre-shifted to the output depth
  __shared__ int tflag[2];                     // per tile parity: some staged code outside the branch-free bound
  __shared__ int offtab[4];                    // +1 corner offsets along r, g, b (H2S_TAGSEL)
  __shared__ unsigned spread_lds[LP ? 256 : 1];   // LP, Morton table order: code c's bits at every third position
  // PQ: E is produced pre-scaled into table-segment units (the x PQ_SEG is
  // folded into the Y'CbCr->R'G'B' constants)
  constexpr int ESC = TRC == 0 || !LP ? PQ_SEG : 1;   // as px_chain

  const int t = threadIdx.x;
  const int lane = t & 63, w = t >> 6;
  const unsigned ntiles = F.nbx * F.nby * F.nframes;
  unsigned tile = (unsigned)fxcd_remap(blockIdx.x, gridDim.x) * (unsigned)F.tpb;
  const unsigned tend = tile + (unsigned)F.tpb < ntiles ? tile + (unsigned)F.tpb : ntiles;

  // ---- prologue: first tile + tables, all issued before any wait ----
  TileGeo geo = tile_geo(F, tile);
  const LaneOfs lofs = lane_ofs(F, t);
  TileRegs cur = tile_load(F, geo, t, lofs);
  const __amdgpu_buffer_rsrc_t req = __builtin_amdgcn_make_buffer_rsrc((void*)F.eq_lut, (short)0, 2 * F.eq_n, 0x00020000);
  const unsigned eq0 = __builtin_amdgcn_raw_buffer_load_b16(req, 2 * t, 0, 0);  // out of range -> 0
  float4 pq0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const bool stage_pq = TRC == 0 || !LP || F.lp_ipt;   // block-uniform
  if (stage_pq && t < PQ_NSEG) {
    const __amdgpu_buffer_rsrc_t rpq = __builtin_amdgcn_make_buffer_rsrc((void*)F.pq_tab, (short)0, 16 * PQ_NSEG, 0x00020000);
    pq0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rpq, 16 * t, 0, 0));
  }
  // codes at the output depth: shift, or bit replication (h2s_expand;
  // rep_rs = 8 - shift, or 31 for a plain shift: the 8-bit code >> 31 = 0)
  if (t < F.eq_n) eq_lds[t] = (uint16_t)((eq0 << F.shift_out) | (eq0 >> F.rep_rs));
  for (int i = t + 256; i < F.eq_n; i += 256) {  // native 10/12-bit tables
    const unsigned v = __builtin_amdgcn_raw_buffer_load_b16(req, 2 * i, 0, 0);
    eq_lds[i] = (uint16_t)((v << F.shift_out) | (v >> F.rep_rs));
  }
  // the first segment (E' < 1/128) marked (cubic FLT_MAX t: 0 at E = 0,
  // > DARK_MARK above) wherever the table is the PQ EOTF (not the CPU chain's
  // HLG table): px_chain's dark re-run evaluates it exactly
  if (stage_pq && t < PQ_NSEG)
    pq_lds[t + 1] = (TRC == 0 || LP) && t == 0 ? make_float4(0.0f, 0.0f, 3.40282347e38f, 0.0f) : pq0;
  if (stage_pq && t == 255) pq_lds[0] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (t < 2) tflag[t] = 0;
  if (t < 3) offtab[t] = t == 0 ? 12 : (t == 1 ? F.og : F.ob);
  if (LP) {
    unsigned x = (unsigned)t;
    x = (x | (x << 8)) & 0x0F00Fu;
    x = (x | (x << 4)) & 0x0C30C3u;
    spread_lds[t] = (x | (x << 2)) & 0x249249u;
  }
  __syncthreads();   // the flags are zero before any thread's first commit sets one
  if (LP && F.lp_ipt) {
    const __amdgpu_buffer_rsrc_t rpi = __builtin_amdgcn_make_buffer_rsrc((void*)F.pqi_tab, (short)0, 16 * PQI_NTAB, 0x00020000);
    for (int i = t; i < PQI_NTAB; i += 256)
      pqi_lds[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rpi, 16 * i, 0, 0));
  }

  // ---- per-lane step geometry: wave w, step s -> 8x8 sub-block
  // (2w + (s&1), s>>1); lane = pixel (quad q = lane>>2 in a 4x4 quad grid,
  // position lane&3 in the quad) ----
  const int qx = (lane >> 2) & 3, qy = lane >> 4, pxl = lane & 1, pyl = (lane >> 1) & 1;
  const int xl = 16 * w + 2 * qx + pxl, yl = 2 * qy + pyl;           // step (0,0) pixel
  const float* ybase = yin + yl * YST + xl;
  // vertical pass (centre siting): 3 x row cy + row cy-1 (top) / cy+1 (bottom)
  const float* h0 = hrow[0] + (qy + 1) * HST + xl;
  const float* h1 = hrow[1] + (qy + 1) * HST + xl;
  const int hb = pyl ? HST : -HST;
  float* csb = csum[0] + qy * CBW + 8 * w + qx;

  // hot constants live in VGPRs for the whole kernel.  Staged samples:
  // luma Y*ys + y_off (+1 on PQ: pq_z's zero segment), chroma centred on its
  // midpoint code (exact), so E = Y' + a*{U,V} takes 4 FMAs
  const float yoff = in_vgpr(F.y_off_c) * (float)ESC + (ESC == PQ_SEG ? 1.0f : 0.0f);
  const float cmid = in_vgpr(F.c_mid);
  const float a_rv = in_vgpr(F.a_rv[1]) * (float)ESC, a_gv = in_vgpr(F.a_gv[1]) * (float)ESC,
              a_gu = in_vgpr(F.a_gu[1]) * (float)ESC, a_bu = in_vgpr(F.a_bu[1]) * (float)ESC;
  const float stride_g = in_vgpr(F.stride_g), stride_b = in_vgpr(F.stride_b);
  const int og = in_vgpr(F.og), ob = in_vgpr(F.ob), ocr = in_vgpr(F.cr), ocg = in_vgpr(F.cg), ocb = in_vgpr(F.cb);
  const float log2_nm1 = in_vgpr(F.log2_nm1), x_max = in_vgpr(F.x_max);
  const float ysc = in_vgpr(F.ys) * (float)ESC;   // zimg depth-conversion scale
  // S6 ordered dither (h2s_dither ORDERED, 8-bit quantiser): this lane's
  // pixel is (xl, yl) mod 8 at every step (tile and step origins are
  // multiples of 8), so its luma offset is one constant
  const float ydq = F.dither ? dither_off(xl, yl) - 0.5f : 0.0f;
  const StepK K{a_rv, a_gv, a_gu, a_bu, stride_g, stride_b, og, ob, ocr, ocg, ocb, log2_nm1, x_max,
                TM == 5 && !LP ? in_vgpr(F.hable_kb) : F.hable_kb, F.c111, rintf(1.0f / F.inv_nm1), offtab,
                LP ? in_vgpr(F.lp_k2) : 0.0f, LP ? in_vgpr(F.lp_k2 + 255.0f) : 0.0f, LP ? F.lp_cy + ydq : 0.0f,
                LP ? in_vgpr(F.lp_k1) : 0.0f};
  gu32* lut8v = LP ? in_vgpr64(F.lut8x) : nullptr;   // (a 64-bit VGPR base: no SGPRs to spill)
  // libplacebo branch: the rgba8 download offset of this lane's pixel at step
  // s (x mod 16 = xl + 8 (s & 1), y mod 16 = yl + 8 ((s >> 1) & 1): tile
  // origins are multiples of 16)
  float qo[4];
#pragma unroll
  for (int i = 0; i < 4; i++)
    qo[i] = LP ? F.lp_qo + (F.lp_dith ? bayer16(xl + 8 * (i & 1), yl + 8 * (i >> 1)) : 0.5f) -
                     (F.lut_off ? 0.0f : F.lp_k2 * F.lp_qs_f)
               : 0.5f;

  // the 8 compute steps of one tile; FB (fast body): no pixel of the tile can
  // reach the exact EOTF path and there is no BICUBIC scratch, so the 8 steps
  // are one straight-line block the scheduler can interleave
  auto steps = [&](const TileGeo& g, auto fast) {
    constexpr bool FB = decltype(fast)::value;
    if constexpr (FB) {
      H2S_MARK("body: fast");
    } else {
      H2S_MARK("body: exact-capable");
    }
    // BT.2390 / spline: this tile's frame curve (dynamic peak: one record per
    // frame, read through the scalar cache; the frame index is block-uniform)
    CurveConsts cv = F;
    if ((TM == 7 || TM == 8 || LP) && F.cv_frames) cv = curve_of(F.cv_frames, g.f);
    if constexpr (LP && TM == 7) {
      // the curve's constants that meet a second scalar operand in an FMA or
      // med3 (one scalar operand per VOP3 on gfx950): in VGPRs once per
      // tile instead of a v_mov per step (libplacebo instances, which have
      // the VGPRs; round 6)
      cv.b_e1b = in_vgpr(cv.b_e1b), cv.b_tb = in_vgpr(cv.b_tb), cv.b_c2 = in_vgpr(cv.b_c2);
      cv.b_lc = in_vgpr(cv.b_lc), cv.b_bk_b = in_vgpr(cv.b_bk_b), cv.b_bk_d = in_vgpr(cv.b_bk_d);
    } else if constexpr (LP && TM == 8) {
      cv.sp_qb_u = in_vgpr(cv.sp_qb_u), cv.sp_pb_u = in_vgpr(cv.sp_pb_u);
      cv.sp_srcmax = in_vgpr(cv.sp_srcmax), cv.sp_umax = in_vgpr(cv.sp_umax);
    }
    const __amdgpu_buffer_rsrc_t lut = __builtin_amdgcn_make_buffer_rsrc((void*)F.lut_yuv, (short)0, F.lut_bytes, 0x00020000);
    // the 2x2 chroma sums of step s (or, BICUBIC, the pixel's Cb, Cr into the
    // frame's 4:4:4 scratch, which k_chroma_bicubic decimates; the scratch
    // has whole tiles of rows: rows past F.H are written, never read)
    auto chroma_out = [&](int s, float oyv, float ozv) {
      if (!FB && F.chr444) {
        const int px = g.px0 + xl + 8 * (s & 1), py = g.py0 + yl + 8 * (s >> 1);
        F.chr444[(long long)py * F.chr_w + px] = make_float2(oyv * F.inv_c56, ozv * F.inv_c56);
        return;
      }
      // chroma: 2x2 sums; the 4 lanes of a quad store the same value
      H2S_MARK("S6 chroma quad sums");
      const int oc = 4 * (s >> 1) * CBW + 4 * (s & 1);
      const float su = quad_sum(oyv), sv = quad_sum(ozv);
      csb[oc] = su;
      csb[oc + CBH * CBW] = sv;
    };
    if constexpr (LP && DBG == 0) {
      if (!F.lut_off) {   // (launch-uniform)
        // The libplacebo branch's product steps, software-pipelined: step s's
        // lut3d table read (a 64 MiB table: its lines come from the L2 or the
        // MALL) is issued, then step s + 1's S1..S4 run, and only then is
        // step s finished (Y'CbCr, eq, the luma code into yin, the chroma
        // sums), so the read's latency hides behind a whole step of VALU work
        // instead of stalling each step (round 6)
        unsigned vp = 0;
#pragma unroll
        for (int s = 0; s <= 8; s++) {
          unsigned vn = 0;
          if (s < 8) {
            const int oy = 8 * (s >> 1) * YST + 8 * (s & 1);
            const int oh = 4 * (s >> 1) * HST + 8 * (s & 1);
            H2S_MARK("S0 step: staged Y, vertical chroma");
            const float ybs = ybase[oy];
            const float U = fmaf(3.0f, h0[oh], h0[oh + hb]);   // x8 upsampled, centred, exact
            const float V = fmaf(3.0f, h1[oh], h1[oh + hb]);
            float r, gg, bl;
            lin_tone<TRC, TM, DESAT, LP, 0, FB>(F, cv, pq_lds, pqi_lds, K, ybs, U, V, [](float, float, float) {},
                                                 r, gg, bl);
            H2S_MARK("S3 encode");
            vn = lp_table_read(F, K, lut8v, spread_lds, r, gg, bl, qo[s & 3]);
          }
          if (s > 0) {
            const int sp = s - 1;
            const float R8 = (float)(vp & 255u), G8 = (float)((vp >> 8) & 255u), B8 = (float)((vp >> 16) & 255u);
            H2S_MARK("S5 Y'CbCr");
            const f3 o = lp_ycbcr(F, K, R8, G8, B8);
            H2S_MARK("S7 eq");
            // luma code (eq applied, shifted) replaces the luma sample this lane read
            reinterpret_cast<unsigned*>(yin)[yl * YST + xl + 8 * (sp >> 1) * YST + 8 * (sp & 1)] = eq_lds[(int)o.x];
            chroma_out(sp, o.y, o.z);
          }
          vp = vn;
        }
        return;
      }
      H2S_MARK("body: lut off");
    }
#pragma unroll
    for (int s = 0; s < 8; s++) {
      const int oy = 8 * (s >> 1) * YST + 8 * (s & 1);   // compile-time LDS offsets
      const int oh = 4 * (s >> 1) * HST + 8 * (s & 1);
      H2S_MARK("S0 step: staged Y, vertical chroma");
      const float ybs = ybase[oy];
      const float U = fmaf(3.0f, h0[oh], h0[oh + hb]);   // x8 upsampled, centred, exact
      const float V = fmaf(3.0f, h1[oh], h1[oh + hb]);
      const long long di = DBG && g.f == 0 && g.py0 + yl + 8 * (s >> 1) < F.H
                               ? (long long)(g.py0 + yl + 8 * (s >> 1)) * F.dbg_w + g.px0 + xl + 8 * (s & 1)
                               : -1;
      float oyv, ozv;
      // luma code (eq applied, shifted) replaces the luma sample this lane read
      reinterpret_cast<unsigned*>(yin)[yl * YST + xl + oy] = px_chain<TRC, TM, DESAT, LP, DBG, FB>(
          F, cv, pq_lds, pqi_lds, eq_lds, lut8v, spread_lds, lut, K, ybs, U, V, di, oyv, ozv, LP ? qo[s & 3] : 0.5f, ydq);
      chroma_out(s, oyv, ozv);   // (BICUBIC: this pixel's Cb, Cr into the 4:4:4 scratch)
    }
  };
  auto mask_in = [&](uint4& a) {   // h2s_lp_p010 TRUNCATE (block-uniform)
    a.x &= F.in_mask2, a.y &= F.in_mask2, a.z &= F.in_mask2, a.w &= F.in_mask2;
  };

  const int pl = __builtin_amdgcn_readfirstlane(t >> 6) & 1, rem = t & 63;   // chroma store role (t < 128)
  const bool cst = t < 128 && !F.chr444;
  for (;;) {
    H2S_MARK("tile: commit, prefetch");
    // ---- commit this tile's registers to LDS ----
    if (F.in_mask2 != 0xFFFFFFFFu) {   // h2s_lp_p010 TRUNCATE (block-uniform)
      mask_in(cur.ya), mask_in(cur.ua);
      cur.uh &= F.in_mask2;
    }
    const float my = stage_luma<YST>(yin, cur.ya, t >> 3, t & 7, ysc, yoff);
    float mc = 0.0f;
    if ((t & 127) < 72) mc = stage_chroma<HST>(hrow[__builtin_amdgcn_readfirstlane(t >> 7)], cur.ua, cur.uh, t & 127, cmid);
    const int par = (int)(tile & 1u);
    if ((my > F.safe_y || mc > F.safe_c)) tflag[par] = 1;
    const TileGeo g = geo;
    const bool more = tile + 1 < tend;   // block-uniform
    if (more) {
      tile_next(F, geo);
      cur = tile_load(F, geo, t, lofs);  // in flight during this tile's compute
    }
    __syncthreads();
    const bool fb = __builtin_amdgcn_readfirstlane(tflag[par]) == 0 && !F.chr444;
    if (t == 0) tflag[par ^ 1] = 0;   // for the next tile: read by every wave of the previous one before this barrier
    if (fb)
      steps(g, std::integral_constant<bool, true>{});
    else
      steps(g, std::integral_constant<bool, false>{});
    H2S_MARK("tile: store");
    __syncthreads();

    // ---- write the tile: 16-byte (u16) / 8-byte (u8) non-temporal stores ----
    put_luma(F, g, read_luma<YST>(F, yin, t >> 3, t & 7), t >> 3, lofs.sy, 0);
    if (cst) put_chroma(F, g, read_chroma(F, csum[0], pl, rem >> 2, rem & 3), pl, rem >> 2, lofs.sc);
    if (!more) break;
    ++tile;
    __syncthreads();   // the store phase has read yin / csum before they are refilled
  }
}


#define FAST_CASES(X) \
  X(0, 4, 0, 0)       \
  X(0, 4, 1, 0)       \
  X(0, 4, 2, 0)       \
  X(0, 5, 0, 0)       \
  X(0, 5, 1, 0)       \
  X(0, 5, 2, 0)       \
  X(0, 6, 0, 0)       \
  X(0, 6, 1, 0)       \
  X(0, 6, 2, 0)       \
  X(0, 7, 0, 0)       \
  X(0, 8, 0, 0)       \
  X(0, 7, 0, 1)       \
  X(0, 8, 0, 1)       \
  X(0, 4, 0, 1)       \
  X(0, 5, 0, 1)       \
  X(0, 6, 0, 1)       \
  X(1, 4, 0, 0)       \
  X(1, 4, 1, 0)       \
  X(1, 4, 2, 0)       \
  X(1, 5, 0, 0)       \
  X(1, 5, 1, 0)       \
  X(1, 5, 2, 0)       \
  X(1, 6, 0, 0)       \
  X(1, 6, 1, 0)       \
  X(1, 6, 2, 0)       \
  X(1, 7, 0, 0)       \
  X(1, 8, 0, 0)       \
  X(1, 7, 0, 1)       \
  X(1, 8, 0, 1)       \
  X(1, 4, 0, 1)       \
  X(1, 5, 0, 1)       \
  X(1, 6, 0, 1)

// one DBG value's instances (0 = product kernels; 1..5 = the debug instance
// for that h2s_stage) of one chain (LPI 0: the CPU chain, 1: the libplacebo
// branch), explicitly instantiated in exactly one .hip each: the two chains'
// product instances compile in their own translation units, so each gets the
// scheduler that measured fastest for it (_build.py SOURCE_FLAGS)
template <int DBG, int LPI>
hipError_t launch_tile(const FastParams& F, int trc, int tm, int desat, dim3 grid, size_t lds, hipStream_t s) {
#define X(T, M, D, L)                                                                       \
  if constexpr (L == LPI) {                                                                 \
    if (trc == T && tm == M && desat == D) {                                                \
      hipLaunchKernelGGL((k_tile<T, M, D, L, DBG>), grid, dim3(256), lds, s, F);            \
      return hipGetLastError();                                                             \
    }                                                                                       \
  }
  FAST_CASES(X)
#undef X
  return hipErrorInvalidValue;
}
#define H2S_TILE_EXTERN(D, L) \
  extern template hipError_t launch_tile<D, L>(const FastParams&, int, int, int, dim3, size_t, hipStream_t);
#define H2S_TILE_INSTANCE(D, L) \
  template hipError_t launch_tile<D, L>(const FastParams&, int, int, int, dim3, size_t, hipStream_t);

}  // namespace h2s

// p2.h -- two int16 trellis metrics in one 32-bit register (packed "SIMD within a register").
//
// The int16 turbo decoder's arithmetic (tdec_body.h, oracle/o_fec.c) is integer adds, subtracts and
// maxima on values bounded well inside int16 (|normalised metric| <= 6138, |candidate| <= 30690 with
// window normalisation, |LLR| <= 26598).  P2 carries the metrics of TWO code blocks -- lo = a code
// block of one 64-lane group, hi = the same lane of a second group of equal K -- so one gfx950 VOP3P
// instruction (v_pk_add_u16 / v_pk_sub_u16 / v_pk_max_i16 / v_pk_min_i16) advances both.  Every value
// the decoder forms stays inside the int16 range, so the wrapping packed ops are exact and the two
// halves reproduce the scalar int16 decoder bit for bit (tdec_p2_body.h).
//
// Device: clang's 2 x short vector type (the compiler folds half swaps into op_sel modifiers).  Host
// (the test emulation, g++): a two-field struct with the same wrapping semantics.
#pragma once
#include <stdint.h>

#include "dl_common.h"

// device pass: the packed-vector implementation; host passes (hipcc's host side, the g++ emulation):
// the struct one
#if defined(__HIP_DEVICE_COMPILE__)
#define MI_P2D __device__
#else
#define MI_P2D
#endif

namespace mi {

using ::fmaxf;   // the float maximum stays visible next to the P2 overload below

#if defined(__HIP_DEVICE_COMPILE__)
typedef short mi_short2 __attribute__((ext_vector_type(2)));
struct P2 {
  mi_short2 v;
};
__device__ inline P2 p2_make(int lo, int hi) { return P2{mi_short2{(short)lo, (short)hi}}; }
__device__ inline P2 p2_splat(int x) { return P2{mi_short2{(short)x, (short)x}}; }
__device__ inline int p2_lo(P2 a) { return a.v.x; }
__device__ inline int p2_hi(P2 a) { return a.v.y; }
__device__ inline uint32_t p2_bits(P2 a) { return __builtin_bit_cast(uint32_t, a.v); }
__device__ inline P2 p2_from_bits(uint32_t u) { return P2{__builtin_bit_cast(mi_short2, u)}; }
__device__ inline P2 operator+(P2 a, P2 b) { return P2{a.v + b.v}; }
__device__ inline P2 operator-(P2 a, P2 b) { return P2{a.v - b.v}; }
__device__ inline P2 fmaxf(P2 a, P2 b) { return P2{__builtin_elementwise_max(a.v, b.v)}; }
__device__ inline P2 p2_min(P2 a, P2 b) { return P2{__builtin_elementwise_min(a.v, b.v)}; }
// saturating add (v_pk_add_i16 with clamp: the same rate as the wrapping add)
__device__ inline P2 p2_adds(P2 a, P2 b) { return P2{__builtin_elementwise_add_sat(a.v, b.v)}; }
#else
struct P2 {
  int16_t lo, hi;
};
inline P2 p2_make(int lo, int hi) { return P2{(int16_t)lo, (int16_t)hi}; }
inline P2 p2_splat(int x) { return P2{(int16_t)x, (int16_t)x}; }
inline int p2_lo(P2 a) { return a.lo; }
inline int p2_hi(P2 a) { return a.hi; }
inline uint32_t p2_bits(P2 a) { return (uint32_t)(uint16_t)a.lo | ((uint32_t)(uint16_t)a.hi << 16); }
inline P2 p2_from_bits(uint32_t u) { return P2{(int16_t)(uint16_t)u, (int16_t)(uint16_t)(u >> 16)}; }
inline P2 operator+(P2 a, P2 b) { return P2{(int16_t)(a.lo + b.lo), (int16_t)(a.hi + b.hi)}; }
inline P2 operator-(P2 a, P2 b) { return P2{(int16_t)(a.lo - b.lo), (int16_t)(a.hi - b.hi)}; }
inline P2 fmaxf(P2 a, P2 b) { return P2{a.lo > b.lo ? a.lo : b.lo, a.hi > b.hi ? a.hi : b.hi}; }
inline P2 p2_min(P2 a, P2 b) { return P2{a.lo < b.lo ? a.lo : b.lo, a.hi < b.hi ? a.hi : b.hi}; }
inline int16_t p2_sat16(int x) { return (int16_t)(x < -32768 ? -32768 : (x > 32767 ? 32767 : x)); }
inline P2 p2_adds(P2 a, P2 b) { return P2{p2_sat16(a.lo + b.lo), p2_sat16(a.hi + b.hi)}; }
#endif
// clamp both halves to [-c, c]
MI_P2D inline P2 p2_clamp(P2 a, int c) { return p2_min(fmaxf(a, p2_splat(-c)), p2_splat(c)); }

// the additive identity / "minus infinity" of a metric type.  Beta (the tail's start, wrapping adds): -16384 can never
// win a maximum against a reachable state (those stay above -6138 - 3 x 2046) and cannot wrap within the three steps
// after which every state is reachable.  Alpha (the trellis start state): -32768 with SATURATING adds on the alpha side
// (tadd_a below), which also keeps the unreachable states out of the LLR maxima of steps 0..2 (tdec_p2_body.h)
template <class T> struct Metric;
template <> struct Metric<float> {
  __host__ __device__ static float zero() { return 0.0f; }
  __host__ __device__ static float ninf() { return -INFINITY; }
  __host__ __device__ static float ninf_alpha() { return -INFINITY; }
};
template <> struct Metric<P2> {
  MI_P2D static P2 zero() { return p2_splat(0); }
  MI_P2D static P2 ninf() { return p2_splat(-16384); }
  MI_P2D static P2 ninf_alpha() { return p2_splat(-32768); }
};
// the adds that take an alpha metric (alpha + gamma, alpha + gamma + beta): plain for the float decoders, saturating
// for P2.  Every reachable value stays inside +-14R = +-28644 (tdec_p2_body.h), where both adds agree bit for bit.
MI_P2D inline float tadd_a(float a, float b) { return a + b; }
MI_P2D inline P2 tadd_a(P2 a, P2 b) { return p2_adds(a, b); }

}  // namespace mi

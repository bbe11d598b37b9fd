// pgmg_real.h — element-type plumbing shared by the level kernels.
//
// Every level kernel is a template on the grid element type T: double (the
// bit-exact default, PGMG_PRECISION_FP64) or float (PGMG_PRECISION_FP32, SURVEY §8 f3:
// half the bytes, parity stated as a tolerance against the fp64 results).  A lane
// always owns a column pair, so a lane moves V2<T> (16 B for double, 8 B for float) per
// row and array.  Norm partial sums are accumulated in double for both types.
#pragma once
#include <hip/hip_runtime.h>

namespace pgmg {

template <class T> struct Vec2;
template <> struct Vec2<double> { using type = double2; };
template <> struct Vec2<float> { using type = float2; };
template <class T> using V2 = typename Vec2<T>::type;

template <class T>
__device__ __forceinline__ V2<T> ldv(const T *p) { return *reinterpret_cast<const V2<T> *>(p); }
template <class T>
__device__ __forceinline__ void stv(T *p, V2<T> v) { *reinterpret_cast<V2<T> *>(p) = v; }
// the same with only element alignment promised (a column pair of an array with an odd
// pitch: the caller's reference-layout grid).  gfx950 under ROCm runs in unaligned-access
// mode, so this is still ONE global_load/store_dwordx4 (dwordx2 for float)
template <class T>
__device__ __forceinline__ V2<T> ldvu(const T *p)
{
    V2<T> v;
    __builtin_memcpy(&v, p, sizeof(v));
    return v;
}
template <class T>
__device__ __forceinline__ void stvu(T *p, V2<T> v) { __builtin_memcpy(p, &v, sizeof(v)); }
template <class T>
__device__ __forceinline__ void stv_nt(T *p, V2<T> v)
{
    typedef T nv2 __attribute__((ext_vector_type(2)));
    nv2 w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<nv2 *>(p));
}
template <class T>
__device__ __forceinline__ V2<T> mk2(T a, T b)
{
    V2<T> v;
    v.x = a;
    v.y = b;
    return v;
}
template <class T> __device__ __forceinline__ V2<T> zero2() { return mk2<T>(T(0), T(0)); }

// An fp32 column pair as a native 2-vector: arithmetic on it selects the packed VOP3P
// instructions (v_pk_add_f32 / v_pk_mul_f32, a subtraction as an add with neg modifiers),
// each element the same IEEE operation as the scalar expression it restates.  The fp32 pass
// moves half the bytes of fp64 for the same per-row work, so its VALU is a larger share of
// its time than fp64's (0.642 -> 0.613 ms per launch at 16385).
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 pk(float2 v) { return pf2{v.x, v.y}; }
__device__ __forceinline__ float2 unpk(pf2 v) { return mk2<float>(v.x, v.y); }

// r*r accumulated in double (identical to r*r for T = double)
template <class T> __device__ __forceinline__ double sq(T r) { return (double)r * (double)r; }
// acc + r*r with one fused multiply-add: the early-exit partial sums are order-dependent
// anyway (parallel reduction), so their rounding is not part of the bitwise contract
template <class T> __device__ __forceinline__ double sqacc(double acc, T r)
{
    return __builtin_fma((double)r, (double)r, acc);
}

// wave64 DPP lane moves: wave_shr:1 (lane i <- lane i-1), wave_shl:1 (lane i <- lane i+1);
// the edge lane receives 0.  bound_ctrl = true: lanes without a source lane read 0, so
// no "old" operand has to be materialised (one v_mov_b32_dpp per dword, no extra move).
__device__ __forceinline__ int dpp_shr_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int dpp_shl_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xF, 0xF, true); }
__device__ __forceinline__ double dpp_shr(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = dpp_shr_i((int)b);
    const int hi = dpp_shr_i((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double dpp_shl(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = dpp_shl_i((int)b);
    const int hi = dpp_shl_i((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float dpp_shr(float v) { return __int_as_float(dpp_shr_i(__float_as_int(v))); }
__device__ __forceinline__ float dpp_shl(float v) { return __int_as_float(dpp_shl_i(__float_as_int(v))); }

// Sum of one double over the 64 lanes of a wave, returned (bitwise identical) in every
// lane.  DPP row_shr:1,2,4,8 (a Hillis-Steele scan inside each row of 16 lanes, VALU
// latency only) then the four row totals read out with v_readlane: ~10 dependent VALU
// ops instead of six __shfl_xor rounds through the LDS crossbar (ds_bpermute, ~100+
// cycles each), which dominated the per-sweep cost of the LDS tail.  All 64 lanes must
// be active.
template <int CTRL> __device__ __forceinline__ double dpp64(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane64(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum(double v)
{
    v += dpp64<0x111>(v);   // row_shr:1
    v += dpp64<0x112>(v);   // row_shr:2
    v += dpp64<0x114>(v);   // row_shr:4
    v += dpp64<0x118>(v);   // row_shr:8  -> lane 16r+15 holds the total of row r
    return (readlane64(v, 15) + readlane64(v, 31)) + (readlane64(v, 47) + readlane64(v, 63));
}

// elements between an allocation's base and element (0,0): column 1 of every row on a
// 128-byte boundary (15 doubles, 31 floats)
template <class T> constexpr int off_elems() { return 128 / (int)sizeof(T) - 1; }
// row pitch in elements: whole 128-byte lines
template <class T> inline int pitch_elems(int N)
{
    const int q = 128 / (int)sizeof(T);
    return (N + q - 1) / q * q;
}

}  // namespace pgmg

// mbots_device.hpp -- device-side building blocks of the MI355X world step.
//
// Float expressions follow the reference's evaluation order (src/sim/sim.cpp)
// and are compiled with -ffp-contract=off so that no FMA contraction changes a
// rounding; sqrtf and '/' are the correctly rounded gfx950 forms (hipcc
// default oclc_correctly_rounded_sqrt_on).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbots {

// host + device: the world-step math shared by the HIP kernels and the CPU
// execution mode (mbots_cpu.cpp), compiled once per side with -ffp-contract=off
#define MB_HD __host__ __device__ __forceinline__

MB_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
MB_HD float u2f(uint32_t x) { return __builtin_bit_cast(float, x); }

// src/sim/types.hpp:13-14, :78-80; src/entry/mgr.cpp:104-113
constexpr int kNumSpecies = 4;
constexpr int kHidden = 16;
constexpr int kSensor = 32;
constexpr int kRays = kSensor + 1;        // 32 pixels + the finder ray
constexpr int kChunksX = 8;
constexpr int kChunksY = 6;
constexpr int kNumChunks = kChunksX * kChunksY;
constexpr int kChunkW = 16;
constexpr int kMaxPkg = 5;
constexpr int kNumPkg = kNumChunks * kMaxPkg;   // 240 food packages per world
constexpr int kFoodCap = 30;                  // totalAllowedFood
constexpr int kMaxCap = 4096;                 // slot capacity bound (kernel classes 128 / 256 / ... / 4096)
constexpr float kLx = 128.0f;                 // 8 chunks * 16 cells * cellDim 1
constexpr float kLy = 96.0f;
// Quat::angleAxis(+-0.1, z) = (cos .05, 0, 0, +-sin .05), correctly rounded.
constexpr float kRotC = 0.99875026039496624f;
constexpr float kRotS = 0.04997916927067833f;

// ---------------------------------------------------------------------------
// Counter RNG: Threefry-2x32-20 (Random123).  Stands in for Madrona's
// rand::split_i / RNG (sim.cpp:1238-1239); KAT-checked in tests.
// ---------------------------------------------------------------------------
MB_HD uint32_t rotl32(uint32_t x, uint32_t r)
{
    return (x << r) | (x >> (32u - r));
}

MB_HD uint2 threefry2x32(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1)
{
    const uint32_t k2 = 0x1BD11BDAu ^ k0 ^ k1;
    uint32_t x0 = c0 + k0, x1 = c1 + k1;
#define MB_R(r) { x0 += x1; x1 = rotl32(x1, r); x1 ^= x0; }
    MB_R(13) MB_R(15) MB_R(26) MB_R(6)  x0 += k1; x1 += k2 + 1u;
    MB_R(17) MB_R(29) MB_R(16) MB_R(24) x0 += k2; x1 += k0 + 2u;
    MB_R(13) MB_R(15) MB_R(26) MB_R(6)  x0 += k0; x1 += k1 + 3u;
    MB_R(17) MB_R(29) MB_R(16) MB_R(24) x0 += k1; x1 += k2 + 4u;
    MB_R(13) MB_R(15) MB_R(26) MB_R(6)  x0 += k2; x1 += k0 + 5u;
#undef MB_R
    return make_uint2(x0, x1);
}

MB_HD float u01(uint32_t bits)
{
    return (float)(bits >> 8) * (1.0f / 16777216.0f);
}

MB_HD int32_t sample_i32(uint32_t bits, int32_t a, int32_t b)
{
    uint32_t range = (uint32_t)(b - a);
    return a + (int32_t)(((uint64_t)bits * (uint64_t)range) >> 32);
}

// ---------------------------------------------------------------------------
// Math shared by the action and sensor phases
// ---------------------------------------------------------------------------
MB_HD float fmin_std(float a, float b) { return (b < a) ? b : a; }
MB_HD float fmax_std(float a, float b) { return (a < b) ? b : a; }

// Sim::getChunkIndex (sim.inl:49-62)
MB_HD int32_t chunk_index(float cx, float cy)
{
    int32_t x = (int32_t)cx, y = (int32_t)cy;
    if (x < 0 || y < 0 || x >= kChunksX || y >= kChunksY) return -1;
    return x + y * kChunksX;
}

// rot.rotateVec({1,0,0}).normalize() for a z-only quaternion (sim.cpp:466-468)
MB_HD void heading(float w, float z, float &dx, float &dy)
{
    float vx = 1.0f - 2.0f * (z * z);
    float vy = 2.0f * (z * w);
    float len = sqrtf(vx * vx + vy * vy);
    dx = vx / len;
    dy = vy / len;
}

// ---------------------------------------------------------------------------
// Sensor output quantisation
// ---------------------------------------------------------------------------
MB_HD uint8_t depth_u8(float t)
{
    if (!(t < 255.0f)) return 255;
    return (uint8_t)(int32_t)t;
}

// ---------------------------------------------------------------------------
// Wave-level helpers (wave64)
// ---------------------------------------------------------------------------
// a wave-uniform value in an SGPR: the compiler cannot prove that the world
// index (threadIdx.x >> 6) or a value loaded at it is uniform, and would keep
// loop bounds in VGPRs (exec-masked loops, per-lane loads)
__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int32_t uniform(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// number of set bits of `mask` strictly below this lane
__device__ __forceinline__ uint32_t rank_below(uint64_t mask)
{
    return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace mbots

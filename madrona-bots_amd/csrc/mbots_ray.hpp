// mbots_ray.hpp -- ray / circle geometry shared by the K1 finder pass and the
// K3b sensor (build spec DESIGN.md 3.6; float expressions identical to
// oracle/mbots_oracle.c, compiled with -ffp-contract=off).
#pragma once

#include "mbots_device.hpp"

namespace mbots {

constexpr int kMaxFood = kFoodCap + 2;        // live packages == currentNumFood <= 30
constexpr uint32_t kOrderFood = 1u;           // object order: wall 0, food 1.., agents 64..
constexpr uint32_t kOrderAgent = 64u;
constexpr uint32_t kNoKey = 0xFFFFFFFFu;

constexpr float kInLo = 0.0f + 0.2f;          // inner arena rectangle (walls, sim.cpp:157-194)
constexpr float kInHiX = 128.0f - 0.2f;
constexpr float kInHiY = 96.0f - 0.2f;

__device__ __forceinline__ float max0(float x) { return x > 0.0f ? x : 0.0f; }
__device__ __forceinline__ float zq(float z) { return __uint_as_float(__float_as_uint(z) & ~0xFFu); }
__device__ __forceinline__ uint32_t zkey(float z, uint32_t order)
{
    return (__float_as_uint(z) & ~0xFFu) | order;
}

// predicates below use non-short-circuit & | so they compile to VALU selects,
// not exec-mask branches; the float operations are the oracle's
__device__ __forceinline__ bool inside_arena(float ox, float oy)
{
    return (ox >= kInLo) & (ox <= kInHiX) & (oy >= kInLo) & (oy <= kInHiY);
}

// wall depth of a ray: exit from the inner rectangle; 0 inside a wall box
__device__ __forceinline__ float wall_z(float ox, float oy, float dx, float dy)
{
    if (!inside_arena(ox, oy)) return 0.0f;
    float tx = __builtin_inff(), ty = __builtin_inff();
    if (dx > 0.0f) tx = (kInHiX - ox) / dx;
    else if (dx < 0.0f) tx = (kInLo - ox) / dx;
    if (dy > 0.0f) ty = (kInHiY - oy) / dy;
    else if (dy < 0.0f) ty = (kInLo - oy) / dy;
    const float t = fmin_std(tx, ty);
    return t == 0.0f ? 0.0f : t;
}

// object at view depth z hides the wall iff z * d < (X - o) per axis: for
// d > 0 z * d < hi - o, for d < 0 z * d > lo - o, i.e. z * |d| < o - lo (IEEE
// products and differences are sign-symmetric, so this is the same predicate)
__device__ __forceinline__ bool beats_wall(float ox, float oy, float dx, float dy, float z)
{
    const bool bx = (dx == 0.0f) | (z * fabsf(dx) < (dx > 0.0f ? kInHiX - ox : ox - kInLo));
    const bool by = (dy == 0.0f) | (z * fabsf(dy) < (dy > 0.0f ? kInHiY - oy : oy - kInLo));
    return inside_arena(ox, oy) & bx & by;
}

__device__ __forceinline__ uint32_t order_of(int nf, int j)
{
    return j < nf ? kOrderFood + (uint32_t)j : kOrderAgent + (uint32_t)(j - nf);
}

// exact predicate of (f, l) on pixel ray k < 32 with offset u; key or kNoKey
__device__ __forceinline__ uint32_t pixel_key(float f, float l, float u, bool fwdk, uint32_t order)
{
    const float A = f * f - 1.0f, B2 = 2.0f * (l * f), C = l * l - 1.0f;
    const float q = (A * u - B2) * u + C;
    const float p = f + u * l;
    // ahead of the camera: p > 0 (forward) / p < 0 (backward), i.e. (+-p) > 0
    const bool hit = (q <= 0.0f) & ((fwdk ? p : -p) > 0.0f);
    const float z = zq(max0(fwdk ? f - 1.0f : -f - 1.0f));
    const bool near = f * f + l * l <= 1.0f;
    const uint32_t key = zkey(near ? 0.0f : z, order);
    return (hit | near) ? key : kNoKey;
}

// pixel_key's hit test for a far pair (f^2 + l^2 > 1, |f| > 1.5: never "near";
// its key is zkey(fwd ? f - 1 : -f - 1, order) on every pixel it hits)
__device__ __forceinline__ bool far_pixel_hit(float f, float l, float u, bool fwdk)
{
    const float A = f * f - 1.0f, B2 = 2.0f * (l * f), C = l * l - 1.0f;
    const float q = (A * u - B2) * u + C;
    const float p = f + u * l;
    return (q <= 0.0f) & ((fwdk ? p : -p) > 0.0f);
}

// the finder ray (u = 0)
__device__ __forceinline__ uint32_t finder_key(float f, float l, uint32_t order)
{
    const float C = l * l - 1.0f;
    const bool hit = (C <= 0.0f) & (f > 0.0f);
    const bool near = f * f + l * l <= 1.0f;
    const uint32_t key = zkey(near ? 0.0f : zq(max0(f - 1.0f)), order);
    return (hit | near) ? key : kNoKey;
}

// live food packages of a world in (chunk, package) order -> put(s, nf, x, y)
// for s in [0, nf); lane c (< 48) holds chunk c's packed record.  Returns nf
// (== currentNumFood <= 30).
template <typename Put>
__device__ __forceinline__ int stage_food_with(uint64_t rec, uint32_t lane, Put put)
{
    const uint32_t live = (uint32_t)(rec >> 40) & 31u;
    const int cnt = __popc(live);
    int off = 0, tot = 0;
#pragma unroll
    for (int bt = 0; bt < 3; ++bt) {
        const uint64_t m = ballot64((cnt >> bt) & 1);
        off += (int)rank_below(m) << bt;
        tot += __popcll(m) << bt;
    }
    const float bx = (float)((lane % kChunksX) * kChunkW);
    const float by = (float)((lane / kChunksX) * kChunkW);
    int s = off;
#pragma unroll
    for (int k = 0; k < kMaxPkg; ++k) {
        if ((live >> k) & 1u) {
            const uint32_t xy = (uint32_t)(rec >> (8 * k)) & 0xFFu;
            if (s < kMaxFood)   // live packages == currentNumFood <= 30
                put(s, min(tot, kMaxFood), (float)(xy & 15u) + bx, (float)(xy >> 4) + by);
            ++s;
        }
    }
    return min(tot, kMaxFood);
}

__device__ __forceinline__ int stage_food(uint64_t rec, uint32_t lane, float2 *obj)
{
    return stage_food_with(rec, lane, [&](int s, int, float x, float y) { obj[s] = make_float2(x, y); });
}

}  // namespace mbots

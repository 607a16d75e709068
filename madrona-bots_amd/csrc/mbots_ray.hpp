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
// a key is the depth's float bits with the low 9 mantissa bits replaced by the
// object order (food 1 + k, agents 64 + slot < 320): 14 mantissa bits of depth
constexpr uint32_t kOrderMask = 0x1FFu;

constexpr float kInLo = 0.0f + 0.2f;          // inner arena rectangle (walls, sim.cpp:157-194)
constexpr float kInHiX = 128.0f - 0.2f;
constexpr float kInHiY = 96.0f - 0.2f;
constexpr float kOutLo = 0.0f - 0.2f;         // the wall boxes' outer faces
constexpr float kOutHiX = 128.0f + 0.2f;
constexpr float kOutHiY = 96.0f + 0.2f;
// rays see only what lies beyond nearSphere from the camera at the agent's
// centre (mgr.cpp:133; attachEntityToView offset {0,0,0}, sim.cpp:221)
constexpr float kNearSphere = 1.1f;
// other agents: discs of agent_render.obj's cross-section in the rays' plane
// (the mesh's z = 0 section: radii 0.910-0.921)
constexpr float kAgentR = 0.92f;
constexpr float kAgentR2 = 0.8464f;           // kAgentR^2

MB_HD float max0(float x) { return x > 0.0f ? x : 0.0f; }
MB_HD float zq(float z) { return u2f(f2u(z) & ~kOrderMask); }
MB_HD uint32_t zkey(float z, uint32_t order)
{
    return (f2u(z) & ~kOrderMask) | order;
}

// Keys of the large capacity classes (512 / 1024 slots: agent orders past
// 511 no longer fit the 9 low bits): the same quantised depth in the high
// word, the order in the low one -- the same lexicographic (depth, order)
// minimum as the 32-bit key wherever both can hold the order, so a world
// renders the same bits in every class.  Key<K>: make / z / order / none.
template <typename K>
struct Key;
template <>
struct Key<uint32_t> {
    static constexpr uint32_t none = kNoKey;
    MB_HD static uint32_t make(float z, uint32_t order) { return zkey(z, order); }
    MB_HD static float z(uint32_t k) { return u2f(k & ~kOrderMask); }
    MB_HD static uint32_t order(uint32_t k) { return k & kOrderMask; }
};
template <>
struct Key<uint64_t> {
    static constexpr uint64_t none = ~0ull;
    MB_HD static uint64_t make(float z, uint32_t order)
    {
        return ((uint64_t)(f2u(z) & ~kOrderMask) << 32) | order;
    }
    MB_HD static float z(uint64_t k) { return u2f((uint32_t)(k >> 32)); }
    MB_HD static uint32_t order(uint64_t k) { return (uint32_t)k; }
};

// ray k's near point in the agent frame, (c, s) = 1.1 (1, u) / sqrt(1 + u^2)
// (c is also the ray parameter s0 of that point along (1, u)), and
// e = 1.1 sqrt(1 + u^2); the oracle's near_pt
struct NearPt {
    float c, s, e;
};
MB_HD NearPt near_pt(float u)
{
    const float n = sqrtf(1.0f + u * u);
    NearPt r;
    r.c = kNearSphere / n;
    r.s = u * r.c;
    r.e = kNearSphere * n;
    return r;
}

// predicates below use non-short-circuit & | so they compile to VALU selects,
// not exec-mask branches; the float operations are the oracle's
MB_HD bool inside_arena(float ox, float oy)
{
    return (ox >= kInLo) & (ox <= kInHiX) & (oy >= kInLo) & (oy <= kInHiY);
}

// inside one of the four wall boxes (sim.cpp:168-180)
MB_HD bool in_wall_box(float x, float y)
{
    const bool xs = (x >= 0.0f) & (x <= 128.0f), ys = (y >= 0.0f) & (y <= 96.0f);
    const bool bx = ((x >= kOutLo) & (x <= kInLo)) | ((x >= kInHiX) & (x <= kOutHiX));
    const bool by = ((y >= kOutLo) & (y <= kInLo)) | ((y >= kInHiY) & (y <= kOutHiY));
    return (bx & ys) | (by & xs);
}

// wall depth of a ray whose near point lies in the inner rectangle: its exit
// from the rectangle along (dx, dy) from the origin
MB_HD float wall_z(float ox, float oy, float dx, float dy)
{
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
MB_HD bool beats_wall(float ox, float oy, float dx, float dy, float z)
{
    const bool bx = (dx == 0.0f) | (z * fabsf(dx) < (dx > 0.0f ? kInHiX - ox : ox - kInLo));
    const bool by = (dy == 0.0f) | (z * fabsf(dy) < (dy > 0.0f ? kInHiY - oy : oy - kInLo));
    return bx & by;
}

// beats_wall for an origin strictly inside the inner rectangle (kInLo < o <
// kInHi on both axes), with lo = kInLo - o and hi = kInHi - o per axis: the
// same predicate without the sign cases -- for d > 0, lo < 0 <= z d; for d < 0,
// z d <= 0 < hi; for d == 0 both hold (z d is a signed zero), as beats_wall's
// d == 0 case; and lo < z d is o - lo > z |d| negated exactly
MB_HD bool beats_wall_in(float lox, float hix, float loy, float hiy, float dx, float dy, float z)
{
    const float zx = z * dx, zy = z * dy;
    return (lox < zx) & (zx < hix) & (loy < zy) & (zy < hiy);
}
MB_HD bool strictly_inside(float ox, float oy)
{
    return (ox > kInLo) & (ox < kInHiX) & (oy > kInLo) & (oy < kInHiY);
}

// where a ray's near point P0 lies: the inner rectangle (the wall is the exit
// from it), inside a wall box (the wall, at s0), or beyond the walls (a miss)
constexpr int kWallInner = 0, kWallBox = 1, kWallNone = 2;
MB_HD int wall_class(float px, float py)
{
    return inside_arena(px, py) ? kWallInner : in_wall_box(px, py) ? kWallBox : kWallNone;
}

MB_HD uint32_t order_of(int nf, int j)
{
    return j < nf ? kOrderFood + (uint32_t)j : kOrderAgent + (uint32_t)(j - nf);
}

// Exact predicate of a radius-R circle at (f, l) on ray (1, u) (fwdk) or
// -(1, u): the line meets it iff q(u) = (A u - 2 l f) u + C <= 0
// (A = f^2 - R^2, C = l^2 - R^2); the ray leaves it beyond the near sphere iff
// the near point lies inside it or the chord's midpoint lies beyond the near
// point (+-p >= e, p = f + u l).  Key (depth f - R, backward -f - R) or kNoKey.
template <typename K = uint32_t>
MB_HD K pixel_key(float f, float l, float u, const NearPt &np, bool fwdk, uint32_t order)
{
    const float A = f * f - kAgentR2, B2 = 2.0f * (l * f), C = l * l - kAgentR2;
    const float q = (A * u - B2) * u + C;
    const float p = f + u * l;
    const float nx = fwdk ? np.c - f : -np.c - f, ny = fwdk ? np.s - l : -np.s - l;
    const bool in0 = nx * nx + ny * ny <= kAgentR2;
    const bool hit = in0 | ((q <= 0.0f) & ((fwdk ? p : -p) >= np.e));
    const K key = Key<K>::make(zq(max0(fwdk ? f - kAgentR : -f - kAgentR)), order);
    return hit ? key : Key<K>::none;
}

// pixel_key's hit test for a far pair (|f| > kCircleFar: the circle lies
// wholly beyond the near sphere, on one side of the camera plane, so in0 is
// false and +-p >= e reduces to +-p > 0 wherever q <= 0; its key is that of
// pixel_key on every pixel it hits)
MB_HD bool far_pixel_hit(float f, float l, float u, bool fwdk)
{
    const float A = f * f - kAgentR2, B2 = 2.0f * (l * f), C = l * l - kAgentR2;
    const float q = (A * u - B2) * u + C;
    const float p = f + u * l;
    return (q <= 0.0f) & ((fwdk ? p : -p) > 0.0f);
}

// the finder ray (u = 0, forward; near point (1.1, 0), e = 1.1): pixel_key's
// expressions at u = 0 (the oracle evaluates the generic form there)
MB_HD NearPt finder_np() { return near_pt(0.0f); }
template <typename K = uint32_t>
MB_HD K finder_key(float f, float l, uint32_t order)
{
    return pixel_key<K>(f, l, 0.0f, finder_np(), true, order);
}

// ---------------------------------------------------------------------------
// Food: the cube_render.obj +-1 box rotated about z by its package's draw
// (sim.cpp:332-341), seen by the horizontal rays as a rotated square (DESIGN.md
// 3.6).  The rotation is kept as the 22-bit quarter-turn fraction of the draw
// (the cube is symmetric under quarter turns); cos / sin are fixed Taylor
// polynomials in plain float operations (host and device libm differ).
// ---------------------------------------------------------------------------
constexpr float kQuarterTurnUnit = 1.57079632679489662f / 4194304.0f;   // (pi/2) 2^-22

MB_HD float2 food_cs(uint32_t q22)
{
    const float w = (float)q22 * kQuarterTurnUnit;
    const float w2 = w * w;
    const float s = w * (1.0f - w2 * (1.0f / 6.0f) *
                                   (1.0f - w2 * (1.0f / 20.0f) *
                                               (1.0f - w2 * (1.0f / 42.0f) *
                                                           (1.0f - w2 * (1.0f / 72.0f) *
                                                                       (1.0f - w2 * (1.0f / 110.0f))))));
    const float c = 1.0f - w2 * 0.5f *
                               (1.0f - w2 * (1.0f / 12.0f) *
                                           (1.0f - w2 * (1.0f / 30.0f) *
                                                       (1.0f - w2 * (1.0f / 56.0f) *
                                                                   (1.0f - w2 * (1.0f / 90.0f) *
                                                                               (1.0f - w2 * (1.0f / 132.0f))))));
    return make_float2(c, s);
}

// A food square in an agent's frame: centre (f, l), unit axes (p, q) and
// (-q, p).  Ray u is the line Y = u X; with S(v) = v.Y - u v.X the corners'
// S are S(centre) +- S(axis 1) +- S(axis 2), so the line meets the square iff
// |l - u f| <= |q - u p| + |p + u q|.  The square spans view depths
// f -+ (|p| + |q|): wholly ahead of the camera plane it is seen by forward rays
// only (mirrored behind); straddling it, by every ray when the origin is
// inside (|m1|, |m2| <= 1, the origin in box coordinates), else on the side of
// the chord, the sign of its slab entry.  Depth (one per object, as the
// discs' f - R): the nearest corner's, max(0, f - (|p| + |q|)) forward.
struct FoodBox {
    float f, l, p, q, ext;
};

MB_HD FoodBox box_setup(float f, float l, float2 cs, float2 h)
{
    FoodBox b;
    b.f = f;
    b.l = l;
    b.p = cs.x * h.x + cs.y * h.y;
    b.q = cs.x * h.y - cs.y * h.x;
    b.ext = fabsf(b.p) + fabsf(b.q);
    return b;
}

MB_HD bool box_line_hit(const FoodBox &b, float u)
{
    return fabsf(b.l - u * b.f) <= fabsf(b.q - u * b.p) + fabsf(b.p + u * b.q);
}

// box_line_hit at u = 0 (the finder ray): for finite operands x - 0 y and
// x + 0 y are x up to the sign of a zero, which fabsf drops
MB_HD bool box_finder_hit(const FoodBox &b)
{
    return fabsf(b.l) <= fabsf(b.q) + fabsf(b.p);
}

// The ray's exit from the square beyond the near sphere, after the line test:
// forward, every slab's upper end >= s0 (the square's X span [f - ext, f + ext]
// bounds the slab interval: wholly past s0 it is a hit, wholly before a miss);
// backward, every slab's lower end <= -s0.  A slab (box coordinate s b - m,
// m1 = f p + l q, m2 = l p - f q, b1 = p + u q, b2 = u p - q) ends past t iff
// m + 1 >= t b (b > 0) / m - 1 <= t b (b < 0) -- multiplied out, no division.
MB_HD bool slab_reaches(float m, float b, float t)
{
    const float tb = t * b;
    return b > 0.0f ? m + 1.0f >= tb : b < 0.0f ? m - 1.0f <= tb : true;
}
MB_HD bool slab_starts_before(float m, float b, float t)
{
    const float tb = t * b;
    return b > 0.0f ? m - 1.0f <= tb : b < 0.0f ? m + 1.0f >= tb : true;
}

// the line test, then the exit beyond the near sphere (s0 = NearPt.c)
MB_HD bool box_hit(const FoodBox &b, float u, bool fwd, float s0)
{
    if (!box_line_hit(b, u)) return false;
    const float zf = fwd ? b.f : -b.f;          // the square's centre along the ray
    if (zf - b.ext >= s0) return true;          // wholly beyond the near point
    if (zf + b.ext < s0) return false;          // wholly before it
    const float m1 = b.f * b.p + b.l * b.q, m2 = b.l * b.p - b.f * b.q;
    const float b1 = b.p + u * b.q, b2 = u * b.p - b.q;
    if (fwd) return (int)slab_reaches(m1, b1, s0) & (int)slab_reaches(m2, b2, s0);
    return (int)slab_starts_before(m1, b1, -s0) & (int)slab_starts_before(m2, b2, -s0);
}

MB_HD float box_z(const FoodBox &b, bool fwd)
{
    return zq(max0(fwd ? b.f - b.ext : -(b.f + b.ext)));
}

// live food packages of a world in (chunk, package) order -> objects [0, nf):
// position and the box's (cos, sin).  Lane c (< 48) holds chunk c's packed
// record and its packages' rotations (prefetched).  Each lane places its chunk's
// packages with their rotation word; then lane s < nf turns object s's word
// into (cos, sin) -- one polynomial per lane instead of one per package of a
// chunk.  Returns nf (== currentNumFood <= 30).
__device__ __forceinline__ int stage_food(uint64_t rec, const uint32_t (&rot)[kMaxPkg], uint32_t lane,
                                          float2 *obj, float2 *frot)
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
            if (s < kMaxFood) {   // live packages == currentNumFood <= 30
                obj[s] = make_float2((float)(xy & 15u) + bx, (float)(xy >> 4) + by);
                frot[s].x = __uint_as_float(rot[k]);
            }
            ++s;
        }
    }
    const int nf = min(tot, kMaxFood);
    wave_sync();
    if ((int)lane < nf) frot[lane] = food_cs(__float_as_uint(frot[lane].x));
    return nf;
}

}  // namespace mbots

// balance.h — wave-level load balancing of the per-lane traversals.
//
// In the persistent path kernel every lane of a wave starts one traversal
// (extension or shadow ray) per iteration and the wave stays in the trace loop
// until its slowest ray is finished.  Measured on C3 (CTL_PROFILE_TRACE build):
// only 33 of 64 lanes are still traversing during an average inner-node step.
//
// Here lanes whose own traversal has ended help the others: at every round
// boundary an idle lane takes the BOTTOM entry (the oldest pushed, i.e. the
// largest pending subtree) of a busy lane's LDS stack and traverses that
// subtree with the same ray.  The donor overwrites the taken slot with the
// stack sentinel, so its own traversal simply ends when it pops down to it.
// Results of all traversals of one ray meet in an LDS slot per ray owner:
// a 64-bit atomic min on (t bits << 32 | triangle) — exactly the wide
// traversal's tie rule (nearest t, then lowest triangle; one instance), so the
// hit does not depend on which lane found it or when.  The winner's (u, v)
// are written after the min.  Any-hit rays stop all their traversals once one
// hit is in the slot.
//
// Only for one-instance scenes with the 4-wide tree (tie_min on): there the
// result of a traversal is order-independent.  The binary reference-order mode
// keeps the per-lane traversal (first-found ties).
#pragma once
#include "traverse.h"

namespace ctl {

// Closest-hit rays donate too (1) or only any-hit rays (0): a stolen far
// subtree of a closest-hit ray is traversed before the near hit that would
// have culled it is known.
#ifndef CTL_BALANCE_CLOSEST
#define CTL_BALANCE_CLOSEST 0
#endif

// Work is handed out once at least this many lanes of the wave are idle.
#ifndef CTL_BALANCE_IDLE
#define CTL_BALANCE_IDLE 1
#endif

// LDS words of the balancing area, after the lane stacks ([entry][thread]).
//   slot  u64[256]     (t bits << 32 | tri) of each owner's ray
//   uv    float2[256]  winner's barycentrics
//   pend  int[256]     traversals of the owner's ray running on other lanes
//   ray   float[12][256] RayLocal of the owner's ray
//   flg   int[256]     any-hit flag of the owner's ray
//   list  int2[256]    per wave: (stolen entry, ray owner) by match rank
constexpr int kBalWords = 512 + 512 + 256 + 12 * 256 + 256 + 512;
constexpr size_t kBalLdsBytes = sizeof(int) * kBalWords;

__device__ __forceinline__ unsigned long long bal_key(float t, uint32_t tri) {
    return ((unsigned long long)(uint32_t)__float_as_int(t) << 32) | tri;
}

// Closest / any hit of this lane's ray (when `has`), traversed by the whole
// wave.  Every lane of the wave must call it (uniform control flow).
template <bool STATS, bool ALPHA>
__device__ __forceinline__ HitRec trace_balanced(const DevScene& S, LaneStack& st, TraceStats* ts, bool has, f3 o,
                                                 f3 d, float tmax, bool anyhit) {
    typedef Traverser<2, STATS, true, true, ALPHA> Tr;
    const int tid = (int)threadIdx.x;
    const int lane = tid & 63;
    const int wbase = tid & ~63;
    const uint64_t ltmask = (1ull << lane) - 1ull;
    int* B = ctl_lds_stack + kExtraLdsOff;
    unsigned long long* slot = reinterpret_cast<unsigned long long*>(B);
    float2* uv = reinterpret_cast<float2*>(B + 512);
    int* pend = B + 1024;
    float* ray = reinterpret_cast<float*>(B + 1280);
    int* flg = B + 1280 + 12 * 256;
    int2* list = reinterpret_cast<int2*>(B + 1280 + 13 * 256);
    const uint32_t inst = ~(uint32_t)S.start_node;

    Tr T;
    bool ownDone = !has, helping = false;
    int owner = tid;   // owner of the ray this lane currently traverses
    int bot = 1;       // lowest stack slot not yet handed away (slot 0: sentinel)
    T.done = true;
    if (has) {
        T.anyhit = anyhit;
        T.init(S, o, d, 0.0f, S.ray_eps, tmax, st, ts);
        slot[tid] = bal_key(tmax, 0xffffffffu);
        uv[tid] = make_float2(0.0f, 0.0f);
        const float r12[12] = {T.cur.ox, T.cur.oy, T.cur.oz, T.cur.dx, T.cur.dy, T.cur.dz,
                               T.cur.idx, T.cur.idy, T.cur.idz, T.cur.oodx, T.cur.oody, T.cur.oodz};
#pragma unroll
        for (int f = 0; f < 12; f++) ray[f * 256 + tid] = r12[f];
        flg[tid] = anyhit ? 1 : 0;
    }
    pend[tid] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();

    for (uint32_t guard = 0;; guard++) {
        // never spin: a wave that has not converged after this many rounds
        // reports the stack-overflow error instead (ok = false on the host)
        if (guard > (1u << 22)) { st.overflow = true; break; }
        if (!T.done) T.round(S, st, ts);

        // finished traversals merge into their ray's slot
        const bool fin = T.done && (helping || !ownDone);
        if (__any(fin)) {
            const int tgt = helping ? owner : tid;
            const unsigned long long k = bal_key(T.h.t, T.h.tri);
            if (fin) atomicMin(&slot[tgt], k);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
            if (fin) {
                if (T.h.tri != 0xffffffffu && slot[tgt] == k) uv[tgt] = make_float2(T.h.u, T.h.v);
                if (helping) atomicSub(&pend[owner], 1);
                else ownDone = true;
                helping = false;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
        }
        // an any-hit ray is finished everywhere once one of its traversals hit
        if (!T.done && T.anyhit && (uint32_t)slot[helping ? owner : tid] != 0xffffffffu) T.done = true;

        // idle lanes take the bottom stack entry of busy lanes
        // (an owner aborted just above merges its own result first)
        const bool idle = T.done && !helping && ownDone;
        const bool donor = !T.done && (CTL_BALANCE_CLOSEST || T.anyhit) && bot < st.sp && bot < kLdsStack;
        const uint64_t im = __ballot(idle), dm = __ballot(donor);
        if (__popcll(im) >= CTL_BALANCE_IDLE && dm != 0) {
            const int n = min(__popcll(im), __popcll(dm));
            if (donor) {
                const int r = __popcll(dm & ltmask);
                if (r < n) {
                    const int e = ctl_lds_stack[bot * kStackBlock + tid];
                    ctl_lds_stack[bot * kStackBlock + tid] = CTL_SENTINEL;
                    bot++;
                    const int ro = helping ? owner : tid;
                    atomicAdd(&pend[ro], 1);
                    list[wbase + r] = make_int2(e, ro);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __builtin_amdgcn_wave_barrier();
            if (idle) {
                const int r = __popcll(im & ltmask);
                if (r < n) {
                    const int2 w = list[wbase + r];
                    helping = true;
                    owner = w.y;
                    T.cur.ox = ray[0 * 256 + owner]; T.cur.oy = ray[1 * 256 + owner]; T.cur.oz = ray[2 * 256 + owner];
                    T.cur.dx = ray[3 * 256 + owner]; T.cur.dy = ray[4 * 256 + owner]; T.cur.dz = ray[5 * 256 + owner];
                    T.cur.idx = ray[6 * 256 + owner]; T.cur.idy = ray[7 * 256 + owner]; T.cur.idz = ray[8 * 256 + owner];
                    T.cur.oodx = ray[9 * 256 + owner]; T.cur.oody = ray[10 * 256 + owner];
                    T.cur.oodz = ray[11 * 256 + owner];
                    // start from the best hit known for this ray, so the tie
                    // test compares against it exactly as one lane would
                    const unsigned long long best = slot[owner];
                    const float2 buv = uv[owner];
                    T.h.t = __int_as_float((int)(best >> 32));
                    T.h.tri = (uint32_t)best;
                    T.h.node = T.h.tri != 0xffffffffu ? inst : 0xffffffffu;
                    T.h.u = buv.x; T.h.v = buv.y;
                    T.anyhit = flg[owner] != 0;
                    T.span_tmin = 0.0f; T.tri_tmin = S.ray_eps;
                    T.level = 1; T.meshSent = 0;
                    T.nodeBase = S.s_wnode_base; T.triBase = S.s_tri_base; T.idxBase = S.s_idx_base;
                    T.triOffset = S.s_tri_offset; T.instIdx = inst;
                    T.resumeLeaves = false;
                    T.leaf2 = 0;
                    T.done = false;
                    st.sp = 0;
                    st.push(CTL_SENTINEL);
                    bot = 1;
                    if (w.x < 0) { T.leafAddr = w.x; T.nodeAddr = CTL_SENTINEL; }
                    else { T.leafAddr = 0; T.nodeAddr = w.x; }
                }
            }
        }
        const bool complete = ownDone && !helping && T.done && pend[tid] == 0;
        if (__all(complete)) break;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    HitRec h;
    const unsigned long long best = slot[tid];
    const float2 buv = uv[tid];
    h.t = __int_as_float((int)(best >> 32));
    h.tri = (uint32_t)best;
    h.node = h.tri != 0xffffffffu ? inst : 0xffffffffu;
    h.u = h.tri != 0xffffffffu ? buv.x : 0.0f;
    h.v = h.tri != 0xffffffffu ? buv.y : 0.0f;
    return h;
}

}  // namespace ctl

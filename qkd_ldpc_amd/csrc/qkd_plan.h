// qkd_plan.h — the check-phase "wave plan": how the E edges of H are laid out
// across 64-lane wavefronts (host code, no HIP; also compiled by the native
// tests).
//
// The reference updates one check at a time (qkd_ldpc_algorithm.cpp:220-243):
// tanh of every incoming message, a left-to-right product over the check's
// bits in ascending order, then one atanh per edge. On gfx950 the check phase
// runs one EDGE per lane: a wave task is a set of whole checks whose edges sit
// on consecutive lanes (a "segment", bits ascending), so each lane computes
// one tanh and one atanh and reads the other factors of its check's product
// from its segment neighbours with cross-lane shuffles, in the reference's
// order. Checks never straddle two tasks.
//
// Packing: tasks are filled by a bounded subset-sum over the degree classes
// so that, where the degree mix allows, all 64 lanes carry an edge (the
// N=10240 code has 4565 checks of degree 6 and 666 of degree 5: 9x6 + 2x5 =
// 64 fills a wave exactly). Lane utilisation = E / (64 * n_tasks).
//
// Idle lanes (and the kPlanPadTasks tasks appended so that kernels may load
// plan words ahead without bounds tests) point at a dummy column i = N, row 0,
// degree 1: a kernel's reads and writes for them land in padding that nothing
// else reads, so the hot loop needs no idle-lane branches. Their plan_chk
// entry is -1.
//
// Packed plan entry of a lane (two uint32 words, the kernels' uint2):
//   word  bits  0..23  bit index i of the edge (N = the dummy column on an idle lane)
//         bits 24..28  position of the check among bit i's checks (ascending), i.e.
//                      the row of the bit-major message store c2b[k][i]
//   seg   bits  0..19  check index j (0 on an idle lane)
//         bits 20..25  first lane of the segment (the check's first edge)
//         bits 26..31  degree - 1 of the check
#pragma once
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace qkdp {

constexpr uint32_t kPlanBitMask = 0xFFFFFFu;
constexpr uint32_t kPlanChkMask = 0xFFFFFu;
constexpr int kPlanMaxBits = (int)kPlanBitMask;    // N must be < this (dummy column N)
constexpr int kPlanMaxChecks = (int)kPlanChkMask + 1;
constexpr int kPlanPadTasks = 128;                 // idle tasks appended to the plan
constexpr int kPlanMaxDegree = 64;                 // check degree: one wavefront
constexpr int kPlanMaxBitDegree = 32;              // bit degree: 5-bit row index

inline uint32_t plan_word(uint32_t bit, uint32_t krow) { return bit | (krow << 24); }
inline uint32_t plan_seg(uint32_t chk, uint32_t start, uint32_t deg) {
    return chk | (start << 20) | ((deg - 1) << 26);
}

struct WavePlan {
    int32_t n_tasks = 0;                 // real tasks; word/chk hold n_tasks + kPlanPadTasks
    std::vector<uint32_t> word;          // [n_tasks*64] bit | row << 24
    std::vector<uint32_t> seg;           // [n_tasks*64] check | start << 20 | (deg-1) << 26
    std::vector<int32_t> chk;            // [n_tasks*64] check of the slot, -1 idle
    std::vector<int32_t> slot_of_edge;   // [E] plan slot of check-CSR edge k
};

// n bits, m checks, check-CSR (cptr[m+1], cidx[E], rows ascending); krow[E] = row of
// each edge in the bit-major store (its position in the bit's ascending check
// list). Degrees must be in [1, 64]. Returns false if a degree is out of range.
inline bool build_wave_plan(int32_t n, int32_t m, const int32_t* cptr, const int32_t* cidx,
                            const int32_t* krow, WavePlan& p) {
    const uint32_t idle = plan_word((uint32_t)n, 0);
    const uint32_t idle_seg = plan_seg(0, 0, 1);
    // degree classes, largest first; checks of a class in ascending order
    std::vector<std::vector<int32_t>> by_deg(kPlanMaxDegree + 1);
    for (int32_t j = 0; j < m; ++j) {
        const int32_t d = cptr[j + 1] - cptr[j];
        if (d < 1 || d > kPlanMaxDegree) return false;
        by_deg[d].push_back(j);
    }
    std::vector<int> degs;
    for (int d = kPlanMaxDegree; d >= 1; --d)
        if (!by_deg[d].empty()) degs.push_back(d);
    std::vector<size_t> next(kPlanMaxDegree + 1, 0);
    const int nc = (int)degs.size();
    const int cap = 64;
    p.word.clear();
    p.seg.clear();
    p.chk.clear();
    p.slot_of_edge.assign(cptr[m], -1);
    int32_t left = m;
    // reach[i][c]: fill c reachable with classes [0, i); take[i][c]: count of class i-1 used
    std::vector<std::vector<int8_t>> reach(nc + 1, std::vector<int8_t>(cap + 1, 0));
    std::vector<std::vector<int8_t>> take(nc + 1, std::vector<int8_t>(cap + 1, 0));
    while (left > 0) {
        for (auto& r : reach) std::fill(r.begin(), r.end(), 0);
        reach[0][0] = 1;
        for (int i = 0; i < nc; ++i) {
            const int d = degs[i];
            const int avail = (int)(by_deg[d].size() - next[d]);
            // (fills c descending: a fill reachable several ways keeps the way
            // with the most of the larger degrees, the first to reach it --
            // ascending, N = 10240 packed 4x6 + 8x5 before 9x6 + 2x5 and ran
            // out of degree-5 checks after 83 tasks: 507 tasks instead of 490)
            for (int c = cap; c >= 0; --c) {
                if (!reach[i][c]) continue;
                // prefer more of the larger degree: highest count first wins the slot
                for (int x = std::min(avail, (cap - c) / d); x >= 0; --x) {
                    const int c2 = c + x * d;
                    if (!reach[i + 1][c2]) {
                        reach[i + 1][c2] = 1;
                        take[i + 1][c2] = (int8_t)x;
                    }
                }
            }
        }
        int best = cap;
        while (best > 0 && !reach[nc][best]) --best;
        // backtrack the counts, then lay the checks out largest degree first
        std::vector<int> cnt(nc, 0);
        for (int i = nc, c = best; i > 0; --i) {
            cnt[i - 1] = take[i][c];
            c -= cnt[i - 1] * degs[i - 1];
        }
        const int32_t task = p.n_tasks++;
        p.word.resize((size_t)p.n_tasks * 64, idle);
        p.seg.resize((size_t)p.n_tasks * 64, idle_seg);
        p.chk.resize((size_t)p.n_tasks * 64, -1);
        int lane = 0;
        for (int i = 0; i < nc; ++i) {
            const int d = degs[i];
            for (int x = 0; x < cnt[i]; ++x) {
                const int32_t j = by_deg[d][next[d]++];
                --left;
                for (int k = 0; k < d; ++k) {
                    const size_t slot = (size_t)task * 64 + lane + k;
                    p.word[slot] = plan_word((uint32_t)cidx[cptr[j] + k], (uint32_t)krow[cptr[j] + k]);
                    p.seg[slot] = plan_seg((uint32_t)j, (uint32_t)lane, (uint32_t)d);
                    p.chk[slot] = j;
                    p.slot_of_edge[cptr[j] + k] = (int32_t)slot;
                }
                lane += d;
            }
        }
        // idle lanes as degree-1 segments of their own (start = the lane): an
        // extrinsic-sum read of row[start + k] then stays beside the lane's
        // neighbours' entries (start 0 put it on the banks of lane 32's and
        // lane 48's reads: ~5 extra LDS cycles per task, tools/lds_stream_model.py)
        for (int l = lane; l < 64; ++l) p.seg[(size_t)task * 64 + l] = plan_seg(0, (uint32_t)l, 1);
    }
    p.word.resize((size_t)(p.n_tasks + kPlanPadTasks) * 64, idle);
    p.seg.resize((size_t)(p.n_tasks + kPlanPadTasks) * 64, idle_seg);
    p.chk.resize((size_t)(p.n_tasks + kPlanPadTasks) * 64, -1);
    return true;
}

}  // namespace qkdp

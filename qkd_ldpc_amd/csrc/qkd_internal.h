// qkd_internal.h — shared definitions of the HIP library (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qkd_ldpc.h"

namespace qkd {

// Threads per decode workgroup: one workgroup decodes one frame at a time.
#ifndef QKD_DECODE_BLOCK
#define QKD_DECODE_BLOCK 1024
#endif
constexpr int kDecodeBlock = QKD_DECODE_BLOCK;
// Second-iteration tanh table (decode.hip): entries per degree pattern are
// 2^(1 + max_dv) sign codes x max_dv rows; the table is used when
// max_dv <= kTab2MaxDv and n_pat * entries <= kTab2MaxEntries.
constexpr int kTab2MaxDv = 3;   // <= the bit phase's unrolled rows (decode.hip kDvUnroll)
constexpr int kTab2MaxEntries = 2048;
constexpr int kFoldTabMaxEntries = 1024;   // speculative fold table (decode_split.hip), 8 B each
constexpr size_t kC2bPad = 64;             // split kernels: slots added to each workgroup's global region
// per-bit arrays of the split kernels (bit_code, bit_pat): rounds of padding
// past the last round, >= the largest bit-phase load batch minus one
constexpr int kBitPadRounds = 4;
__host__ __device__ inline int tab2_stride(int max_dv) { return (1 << (1 + max_dv)) * max_dv; }

// Largest check degree: one check's edges fit one wavefront (qkd_plan.h).
constexpr int kMaxCheckDegree = 64;
// The per-frame bit totals live in LDS as binary64: N <= this.
constexpr int kMaxBitsLds = 20480;
// The split-store kernels (decode_split.hip): Bob's bits of a thread's
// bit-phase rounds in one 64-bit register, 64 rounds of kDecodeBlock bits
constexpr int kMaxBitsSplit = 64 * kDecodeBlock;
// longer codes (the frame-interleaved decoder and its exact hand-off kernel,
// decode_split_kernel<..., LONG>): the split view's arrays exist up to this
constexpr int kMaxBitsSplitLong = 128 * kDecodeBlock;
// (the split decoder's encoded segment words hold (j >> 5) * 4 in 13 bits:
// qkd_decode.h encode_seg)
constexpr int32_t kMaxChecksSplit = 65536;
// Parallel key generation: 64 lanes per frame, jump levels log2(64); frames
// with more flipped positions than this take the serial kernel.
// keygen_fast_kernel: kKeygenLanes lanes per frame (kKeygenLevels = log2 of
// it jump levels), kKeygenFrames frames per workgroup of kKeygenBlock threads
#ifndef QKD_KEYGEN_LEVELS
#define QKD_KEYGEN_LEVELS 6
#endif
constexpr int kKeygenLevels = QKD_KEYGEN_LEVELS;
constexpr int kKeygenLanes = 1 << kKeygenLevels;
constexpr int kKeygenBlock = kKeygenLanes < 64 ? 64 : kKeygenLanes;   // threads per workgroup
constexpr int kKeygenFrames = kKeygenBlock / kKeygenLanes;
constexpr uint32_t kKeygenFastMaxErrors = 4096;
// keygen_split_kernel: lanes per frame in each of its two waves (Alice's bits,
// shuffle draws), so 64 / kKgSplitLanes frames per 128-thread workgroup
#ifndef QKD_KG_SPLIT_LANES
#define QKD_KG_SPLIT_LANES 64
#endif
constexpr uint32_t kKgSplitLanes = QKD_KG_SPLIT_LANES;
// wave pairs (one Alice wave, one shuffle wave) per workgroup
#ifndef QKD_KG_PAIRS
#define QKD_KG_PAIRS 1
#endif
constexpr uint32_t kKgPairs = QKD_KG_PAIRS;
constexpr uint32_t kKgBlock = 128 * kKgPairs;
constexpr uint32_t kKgSplitFrames = kKgPairs * (64 / kKgSplitLanes);
static_assert(kKgSplitLanes >= 1 && 64 % kKgSplitLanes == 0, "lanes per frame divide a wave");

// Device-resident, immutable view of H.
//   chk_bits[k * m_pad + j]  bit index of slot k of check j (ascending), -1 pad
//                            (thread-per-check syndrome kernel)
//   plan[s]                  the check-phase wave plan (qkd_plan.h): slot
//                            s = task*64 + lane holds one edge: {bit | row,
//                            check | segment start | degree} (qkd_plan.h)
//   bit_chk[k * n_pad + i]   k-th check of bit i (ascending), -1 pad
//   bit_pos[k * n_pad + i]   position of bit i in that check's ascending row
//                            (LDS min-sum state lookups)
// Slot-major ("ELL") layouts keep lane-consecutive bits on consecutive
// addresses.
struct DeviceCode {
    int32_t n, m, e;
    int32_t n_pad, m_pad;
    int32_t max_dv, max_dc, min_dc;
    int32_t min_dv;
    int32_t n_tasks;
    const int32_t* chk_bits;
    const uint8_t* chk_deg;
    const uint2* plan;            // {bit | row << 24, check | start << 20 | (deg-1) << 26}
    const int32_t* bit_chk;
    const uint8_t* bit_pos;
    const uint8_t* bit_deg;
    // degree patterns of the bits (second-iteration tanh table, decode.hip):
    // bit_pat[i] = pattern of bit i; pat_deg[p * max_dv + k] = degree of the
    // k-th check of pattern p (0 past the bit's degree)
    int32_t n_pat;
    const uint16_t* bit_pat;
    const uint8_t* pat_deg;
    // packed per-bit word (speculative bit phases; nullptr unless M <= 65536,
    // bit degree <= 3 and check degree <= 16): bits 0-15 / 16-31 / 32-47 the
    // bit's checks in ascending order (0 past its degree), 48-49 its degree,
    // 50-53 / 54-57 / 58-61 each check's degree - 1
    const uint64_t* bit_code;
    // plan with the message slot row * n_pad + bit in place of {bit, row}
    // (split kernels: their message store is slot-addressed)
    const uint2* plan_slot;
    // The split kernels' view (qkd_code::view_split) numbers bits in an
    // internal order (host.cpp build_code): bit_chk, bit_deg, bit_pat,
    // bit_code and plan_slot are indexed by internal bit q, whose original
    // bit is perm[q]; inv[bit] = q. nullptr in the classic kernels' view
    // (original order). bit_code and plan_slot exist in the internal order only.
    const int32_t* perm;
    const int32_t* inv;
    // frame_syn_sliced_kernel (split view, N < 65535, check degree <= 16;
    // else nullptr): chk_rows16[j * chk_rs + k] = bit k of check j (0xffff
    // past the row; chk_rs 8 or 16)
    const uint16_t* chk_rows16;
    int32_t chk_rs;
    // the frame-interleaved decoder (decode_ilv.hip; split view, bit_code
    // present, check degree <= 16): ilv_slots[j * ilv_rs + k] = the message
    // line (row * n_pad + internal bit) of the k-th edge of check j, ~0 past
    // its degree (ilv_rs 8 or 16); nullptr otherwise
    const uint32_t* ilv_slots;
    int32_t ilv_rs;
    // chk_odd[w] bit b = deg(check 32 w + b) & 1, in the split kernels'
    // syndrome-word layout (decode_m_words words; the keys path's running
    // syndrome starts from it, decode_split.hip)
    const uint32_t* chk_odd;
};

}  // namespace qkd

// the speculation policy's record of one QBER (decode.hip decode_keys): clean =
// consecutive replay samples under the switch; skip = calls since the last
// sample once clean >= 2 (sampled every kSpecStatEvery calls)
struct SpecClean {
    int clean = 0;
    uint64_t skip = 0;
};

struct qkd_workspace {
    const qkd_code* code = nullptr;
    int device = 0;
    std::mutex mu;
    // qkd_debug_set_option values of this workspace (host.cpp debug_option)
    std::map<std::string, std::string> dbg;
    // decode scratch: one c2b region per resident workgroup
    double* c2b = nullptr;
    size_t c2b_slots = 0;
    // dynamic frame queue counter (zeroed per launch)
    uint32_t* counter = nullptr;
    // packed alice / bob keys (uint64 words) for the fused paths
    uint64_t* alice_w = nullptr;
    uint64_t* bob_w = nullptr;
    size_t key_frames = 0;
    // split decoder, keys path (decode_split.hip): per frame the target and
    // first-product syndrome words (frame_syn_kernel) and the hard decision
    // words the decoder leaves for key_match_kernel; sized with the keys
    uint32_t* synw = nullptr;
    uint64_t* zout = nullptr;
    // keygen shuffle scratch (ne words per frame)
    uint32_t* low = nullptr;
    size_t low_words = 0;
    hipEvent_t done = nullptr;
    // speculation policy across calls (decode.hip, decode_keys): the replay
    // count of the last speculative call comes back asynchronously; a QBER
    // point whose frames were replayed too often (kSpecCkptSwitch) switches it
    // and every higher QBER on this workspace to the checkpointed speculation
    uint32_t* spec_stat_host = nullptr;     // pinned: replays of the last call
    hipEvent_t spec_stat_ev = nullptr;
    bool spec_stat_pending = false;
    double spec_stat_q = 0.0;
    size_t spec_stat_frames = 0;
    double spec_ckpt_q = 2.0;
    // per QBER: consecutive samples under the switch (decode_keys samples a
    // QBER with two such samples only every kSpecStatEvery calls)
    std::map<double, SpecClean> spec_clean;
    // checkpointed speculation: one saved message store per resident workgroup
    double* ckpt = nullptr;
    size_t ckpt_slots = 0;
    // the speculative kernel's in-launch policy windows (DecodeArgs::win)
    uint32_t* win = nullptr;
    size_t win_words = 0;
    // the frame-interleaved decoder (decode_ilv.hip): message lines of every
    // resident workgroup (16 frames per 128-byte line), and the frames it
    // hands to the split kernel's exact replays
    double* ilv = nullptr;
    size_t ilv_elems = 0;
    uint32_t* fb_list = nullptr;
    size_t fb_frames = 0;
    // qkd_debug_decoder_timing: while on, HIP events bracket every decoder
    // launch on its stream (pairs recorded, read back on collection)
    bool time_decoder = false;
    std::vector<hipEvent_t> dec_ev;        // start, stop, start, stop, ...
    size_t dec_ev_used = 0;
    double dec_ms_folded = 0.0;            // finished pairs folded in (pool bound)
    uint64_t dec_pairs_folded = 0;
};

struct qkd_code {
    int device = 0;
    int32_t n = 0, m = 0, e = 0;
    int32_t max_dv = 0, max_dc = 0, min_dc = 0, min_dv = 0, is_regular = 0;
    int32_t n_pad = 0, m_pad = 0;
    int32_t n_tasks = 0;
    std::vector<int32_t> check_ptr, check_idx, bit_ptr, bit_idx;
    int32_t* d_chk_bits = nullptr;
    uint8_t* d_chk_deg = nullptr;
    int32_t* d_bit_chk = nullptr;
    uint8_t* d_bit_pos = nullptr;
    uint8_t* d_bit_deg = nullptr;
    uint2* d_plan = nullptr;
    uint2* d_plan_slot = nullptr;
    // the slot plan on the host, and its encoded forms by LDS layout
    // ((S, message base) -> device copy, qkd::plan_for_layout; plan_mu guards
    // the map: workspaces on several threads may share the code)
    std::vector<uint2> plan_slot_host;
    mutable std::map<std::pair<uint32_t, uint32_t>, uint2*> d_plan_enc;
    mutable std::mutex plan_mu;
    int32_t n_pat = 0;                  // 0: too many degree patterns for the table
    std::vector<uint8_t> pat_deg;
    uint16_t* d_bit_pat = nullptr;
    uint64_t* d_bit_code = nullptr;
    uint8_t* d_pat_deg = nullptr;
    // the split kernels' internal bit order (DeviceCode::perm / inv) and the
    // per-bit arrays in it
    int32_t* d_perm = nullptr;
    int32_t* d_inv = nullptr;
    // frame_syn_sliced_kernel's compact check rows (host.cpp)
    uint16_t* d_chk_rows16 = nullptr;
    int32_t chk_rs = 0;
    uint32_t* d_ilv_slots = nullptr;
    int32_t ilv_rs = 0;
    uint32_t* d_chk_odd = nullptr;
    int32_t* d_bit_chk_s = nullptr;
    uint8_t* d_bit_deg_s = nullptr;
    uint16_t* d_bit_pat_s = nullptr;
    // parallel key generation (decode.hip: keygen_fast_kernel): lane l of a
    // frame's kKeygenLanes-lane slice starts at draw l * keygen_chunk;
    // d_jump[b] = T^(chunk * 2^b)
    uint32_t keygen_chunk = 0;
    uint64_t* d_jump = nullptr;
    // the same jumps as polynomials: d_jpoly[l] = x^(l * chunk) mod P (4 words)
    uint64_t* d_jpoly = nullptr;
    // keygen_split_kernel (the default): a frame's lane l of wave 0 draws
    // Alice's bits [l * kg_cb, (l + 1) * kg_cb), its lane l of wave 1 the
    // shuffle draws from N + l * kg_cs; d_jpoly2[w * kKgSplitLanes + l] =
    // x^(start) mod P
    uint32_t kg_cb = 0, kg_cs = 0;
    uint64_t* d_jpoly2 = nullptr;
    int cu_count = 0;
    qkd_workspace* default_ws = nullptr;

    // the classic kernels' view (original bit order)
    qkd::DeviceCode view() const {
        return qkd::DeviceCode{n, m, e, n_pad, m_pad, max_dv, max_dc, min_dc, min_dv, n_tasks,
                               d_chk_bits, d_chk_deg, d_plan, d_bit_chk, d_bit_pos, d_bit_deg,
                               n_pat, d_bit_pat, d_pat_deg, nullptr, nullptr, nullptr, nullptr,
                               nullptr, 0, nullptr, 0, d_chk_odd};
    }
    // the split kernels' view (internal bit order, DeviceCode::perm)
    qkd::DeviceCode view_split() const {
        return qkd::DeviceCode{n, m, e, n_pad, m_pad, max_dv, max_dc, min_dc, min_dv, n_tasks,
                               d_chk_bits, d_chk_deg, d_plan, d_bit_chk_s, nullptr, d_bit_deg_s,
                               n_pat, d_bit_pat_s, d_pat_deg, d_bit_code, d_plan_slot, d_perm, d_inv,
                               d_chk_rows16, chk_rs, d_ilv_slots, ilv_rs, d_chk_odd};
    }
};

namespace qkd {

qkd_status set_error(qkd_status s, const char* fmt, ...);
void clear_error();

// A debug / A-B option (qkd_debug_set_option, host.cpp): the workspace's
// value, else the process-wide one, else unset (the product behaviour). The
// library reads no environment variable.
struct DbgOpt {
    bool set = false;
    std::string v;
    explicit operator bool() const { return set; }
    const char* c_str() const { return v.c_str(); }
    int as_int() const { return atoi(v.c_str()); }
    long as_long() const { return atol(v.c_str()); }
    bool is(const char* s) const { return set && v == s; }
};
DbgOpt debug_option(const qkd_workspace* ws, const char* name);

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

#define QKD_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return ::qkd::set_error(QKD_ERR_DEVICE, "%s failed: %s (%s:%d)", #call,       \
                                    hipGetErrorString(e_), __FILE__, __LINE__);           \
    } while (0)

// Workspace helpers (decode.hip).
qkd_status ws_reserve_decode(qkd_workspace* ws, size_t slots);
qkd_status ws_reserve_keys(qkd_workspace* ws, size_t frames, size_t low_words);
qkd_workspace* resolve_ws(const qkd_code* code, qkd_workspace* ws);

}  // namespace qkd

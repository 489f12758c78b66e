// host.cpp — code objects, matrix readers, errors and host helpers of the
// C ABI (include/qkd_ldpc.h). Device kernels live in decode.hip.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <new>
#include <sstream>

#include "qkd_internal.h"
#include "qkd_plan.h"
#include "qkd_rng.h"

namespace qkd {

static thread_local std::string g_last_error;

qkd_status set_error(qkd_status s, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return s;
}

void clear_error() { g_last_error.clear(); }

// ---- debug / A-B options (qkd_debug_set_option) -----------------------------
static const char* const kDebugOptions[] = {
    "QKD_SPEC_CAP", "QKD_SPEC_CKPT", "QKD_CKPT_UNSAT", "QKD_SPEC_POLICY", "QKD_FOLD_TABLE",
    "QKD_DECODE_KERNEL", "QKD_MINSUM_STORE", "QKD_DECODE_GRID", "QKD_SPLIT_BUDGET", "QKD_C2B_PAD",
    "QKD_ILV", "QKD_ILV_GRID", "QKD_KEYGEN", "QKD_SYN_SLICED", "QKD_SYN_BYTES", "QKD_BIT_ORDER",
    "QKD_PHASE_TIMING"};
static std::mutex g_dbg_mu;                            // guards g_dbg and every workspace's dbg
static std::map<std::string, std::string> g_dbg;

DbgOpt debug_option(const qkd_workspace* ws, const char* name) {
    std::lock_guard<std::mutex> lock(g_dbg_mu);
    DbgOpt o;
    if (ws) {
        const auto it = ws->dbg.find(name);
        if (it != ws->dbg.end()) {
            o.set = true;
            o.v = it->second;
            return o;
        }
    }
    const auto it = g_dbg.find(name);
    if (it != g_dbg.end()) {
        o.set = true;
        o.v = it->second;
    }
    return o;
}

static int32_t round_up(int32_t x, int32_t a) { return (x + a - 1) / a * a; }

static void free_device(qkd_code* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->d_chk_bits) (void)hipFree(c->d_chk_bits);
    if (c->d_chk_deg) (void)hipFree(c->d_chk_deg);
    if (c->d_bit_chk) (void)hipFree(c->d_bit_chk);
    if (c->d_bit_pos) (void)hipFree(c->d_bit_pos);
    c->d_bit_pos = nullptr;
    if (c->d_bit_deg) (void)hipFree(c->d_bit_deg);
    if (c->d_bit_pat) (void)hipFree(c->d_bit_pat);
    if (c->d_bit_code) (void)hipFree(c->d_bit_code);
    c->d_bit_code = nullptr;
    if (c->d_pat_deg) (void)hipFree(c->d_pat_deg);
    for (void* p : {(void*)c->d_perm, (void*)c->d_inv, (void*)c->d_bit_chk_s, (void*)c->d_bit_deg_s,
                    (void*)c->d_bit_pat_s, (void*)c->d_chk_rows16, (void*)c->d_ilv_slots, (void*)c->d_chk_odd})
        if (p) (void)hipFree(p);
    c->d_chk_odd = nullptr;
    c->d_chk_rows16 = nullptr;
    c->chk_rs = 0;
    c->d_ilv_slots = nullptr;
    c->ilv_rs = 0;
    c->d_perm = c->d_inv = c->d_bit_chk_s = nullptr;
    c->d_bit_deg_s = nullptr;
    c->d_bit_pat_s = nullptr;
    c->d_bit_pat = nullptr;
    c->d_pat_deg = nullptr;
    if (c->d_plan) (void)hipFree(c->d_plan);
    c->d_plan = nullptr;
    if (c->d_plan_slot) (void)hipFree(c->d_plan_slot);
    c->d_plan_slot = nullptr;
    for (auto& kv : c->d_plan_enc) (void)hipFree(kv.second);
    c->d_plan_enc.clear();
    if (c->d_jump) (void)hipFree(c->d_jump);
    c->d_jump = nullptr;
    if (c->d_jpoly) (void)hipFree(c->d_jpoly);
    c->d_jpoly = nullptr;
    if (c->d_jpoly2) (void)hipFree(c->d_jpoly2);
    c->d_jpoly2 = nullptr;
    c->d_chk_bits = nullptr;
    c->d_chk_deg = nullptr;
    c->d_bit_chk = nullptr;
    c->d_bit_deg = nullptr;
}

// The internal order's second pass (build_code): inside each task's run of
// last-row bits the order is free (the run stays one run of slots), and it
// decides the LDS banks of the OTHER rows' slots of those bits, which the
// check phases read and write scattered: slot x = row * n_pad + bit sits in
// the bank pair x mod 32 (8-byte slots over 64 four-byte banks), and a
// half-wave's accesses serialise on the busiest pair. A deterministic local
// search swaps bits within runs while the summed excess over the tasks'
// half-waves (busiest pair's count - 1, not-last-row edges) does not grow
// (tools/bank_model.py: 3.06 -> ~1.1 extra bank cycles per task for the
// N = 10240 code).
static void bank_balance_runs(int32_t n, int32_t n_pad, const std::vector<int32_t>& bdeg,
                              const qkdp::WavePlan& plan, std::vector<int32_t>& perm, std::vector<int32_t>& inv) {
    const int32_t n_tasks = plan.n_tasks;
    std::vector<std::vector<int32_t>> tasks_of(n);
    std::vector<std::vector<int32_t>> runs(n_tasks);
    for (int32_t t = 0; t < n_tasks; ++t)
        for (int l = 0; l < 64; ++l) {
            const uint32_t w = plan.word[(size_t)t * 64 + l];
            const uint32_t b = w & qkdp::kPlanBitMask;
            if (b >= (uint32_t)n) continue;
            if ((int32_t)(w >> 24) == bdeg[b] - 1) runs[t].push_back((int32_t)b);
            if (tasks_of[b].empty() || tasks_of[b].back() != t) tasks_of[b].push_back(t);
        }
    // (the edges of a task are distinct slots; idle lanes are skipped)
    auto cost = [&](int32_t t) {
        int ex = 0;
        for (int h = 0; h < 2; ++h) {
            int cnt[32] = {0};
            for (int l = h * 32; l < h * 32 + 32; ++l) {
                const uint32_t w = plan.word[(size_t)t * 64 + l];
                const uint32_t b = w & qkdp::kPlanBitMask;
                const int32_t row = (int32_t)(w >> 24);
                if (b >= (uint32_t)n || row == bdeg[b] - 1) continue;
                cnt[((uint32_t)row * (uint32_t)n_pad + (uint32_t)inv[b]) & 31u]++;
            }
            int mx = 0;
            for (int k = 0; k < 32; ++k) mx = std::max(mx, cnt[k]);
            ex += mx > 0 ? mx - 1 : 0;
        }
        return ex;
    };
    std::vector<int> cur(n_tasks);
    for (int32_t t = 0; t < n_tasks; ++t) cur[t] = cost(t);
    uint64_t rng = 0x9e3779b97f4a7c15ull;
    auto next = [&]() {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    const int64_t iters = std::min<int64_t>(200000, (int64_t)20 * n);
    std::vector<int32_t> aff;
    std::vector<int> nc;
    for (int64_t it = 0; it < iters; ++it) {
        const auto& run = runs[next() % (uint64_t)n_tasks];
        if (run.size() < 2) continue;
        const int32_t a = run[next() % run.size()], b = run[next() % run.size()];
        if (a == b) continue;
        aff.clear();
        for (int32_t t : tasks_of[a]) aff.push_back(t);
        for (int32_t t : tasks_of[b]) aff.push_back(t);
        std::sort(aff.begin(), aff.end());
        aff.erase(std::unique(aff.begin(), aff.end()), aff.end());
        int before = 0;
        for (int32_t t : aff) before += cur[t];
        std::swap(inv[a], inv[b]);
        int after = 0;
        nc.resize(aff.size());
        for (size_t k = 0; k < aff.size(); ++k) after += nc[k] = cost(aff[k]);
        if (after <= before) {
            for (size_t k = 0; k < aff.size(); ++k) cur[aff[k]] = nc[k];
        } else {
            std::swap(inv[a], inv[b]);
        }
    }
    for (int32_t i = 0; i < n; ++i) perm[inv[i]] = i;
}

// The split kernels' internal bit order (decode_split.hip, DeviceCode::perm):
// bits numbered in the order the check-phase plan meets their LAST edge (row
// deg - 1), task by task, lane by lane. Each task's last-row edges then have
// consecutive internal bits, and so consecutive message slots (row * n_pad +
// bit): the last row is the one the split store keeps in global memory, so a
// check phase's global accesses come in runs of whole lines instead of one
// line per edge, while the bit phase, which walks the internal order, stays
// coalesced. Then bank_balance_runs orders each run for the LDS banks.
// perm[internal] = bit, inv[bit] = internal; bits without edges go last.
// mode (diagnostics, QKD_BIT_ORDER): "identity" keeps the original order,
// "runs" skips the bank pass.
static void internal_bit_order(int32_t n, int32_t n_pad, const std::vector<int32_t>& bdeg,
                               const qkdp::WavePlan& plan, std::vector<int32_t>& perm, std::vector<int32_t>& inv,
                               const char* mode) {
    int32_t nx = 0;
    for (size_t k = 0; k < (size_t)plan.n_tasks * 64; ++k) {
        const uint32_t b = plan.word[k] & qkdp::kPlanBitMask;
        if (b < (uint32_t)n && (int32_t)(plan.word[k] >> 24) == bdeg[b] - 1 && inv[b] < 0) {
            inv[b] = nx;
            perm[nx++] = (int32_t)b;
        }
    }
    for (int32_t i = 0; i < n; ++i)
        if (inv[i] < 0) {
            inv[i] = nx;
            perm[nx++] = i;
        }
    if (mode && !strcmp(mode, "identity")) {
        for (int32_t i = 0; i < n; ++i) perm[i] = inv[i] = i;
    } else if (!(mode && !strcmp(mode, "runs"))) {
        bank_balance_runs(n, n_pad, bdeg, plan, perm, inv);
    }
}

// The check-side CSR's invariants (qkd_code_create): cptr[0] = 0, monotone
// offsets, at least one edge, bit indices in range, every row strictly
// ascending (QKD_ERR_UNSORTED when a row descends: the reference would
// silently mis-route its messages). Fills bdeg[n] (bit
// degrees) and max_dc.
static qkd_status validate_csr(int32_t n, int32_t m, const int32_t* cptr, const int32_t* cidx,
                               std::vector<int32_t>& bdeg, int32_t& max_dc) {
    if (n <= 0 || m <= 0 || !cptr || !cidx)
        return set_error(QKD_ERR_INVALID_ARG, "qkd_code_create: n=%d m=%d, null adjacency", n, m);
    if (cptr[0] != 0) return set_error(QKD_ERR_BAD_CODE, "check_ptr[0] must be 0");
    for (int32_t j = 0; j < m; ++j)
        if (cptr[j + 1] < cptr[j])
            return set_error(QKD_ERR_BAD_CODE, "check_ptr not monotone at check %d", j);
    if (cptr[m] <= 0) return set_error(QKD_ERR_BAD_CODE, "code has no edges");
    max_dc = 0;
    bdeg.assign(n, 0);
    for (int32_t j = 0; j < m; ++j) {
        const int32_t d = cptr[j + 1] - cptr[j];
        max_dc = std::max(max_dc, d);
        for (int32_t k = cptr[j]; k < cptr[j + 1]; ++k) {
            const int32_t b = cidx[k];
            if (b < 0 || b >= n)
                return set_error(QKD_ERR_BAD_CODE, "check %d: bit index %d out of range [0,%d)", j, b, n);
            if (k > cptr[j] && cidx[k - 1] >= b)
                return set_error(cidx[k - 1] == b ? QKD_ERR_BAD_CODE : QKD_ERR_UNSORTED,
                                 "check %d: bit list not strictly ascending at slot %d (%d after %d)",
                                 j, k - cptr[j], b, cidx[k - 1]);
            bdeg[b]++;
        }
    }
    return QKD_OK;
}

// Validate the check-side CSR, derive the bit side, upload the ELL layouts.
static qkd_status build_code(qkd_code* c, int32_t n, int32_t m, const int32_t* cptr,
                             const int32_t* cidx, int device) {
    std::vector<int32_t> bdeg;
    int32_t max_dc = 0;
    qkd_status vs = validate_csr(n, m, cptr, cidx, bdeg, max_dc);
    if (vs != QKD_OK) return vs;
    const int32_t e = cptr[m];
    int32_t max_dv = 0;
    for (int32_t i = 0; i < n; ++i) max_dv = std::max(max_dv, bdeg[i]);
    if (max_dc > kMaxCheckDegree)
        return set_error(QKD_ERR_UNSUPPORTED, "check degree %d exceeds %d", max_dc, kMaxCheckDegree);
    if (max_dv > qkdp::kPlanMaxBitDegree)
        return set_error(QKD_ERR_UNSUPPORTED, "bit degree %d exceeds %d", max_dv, qkdp::kPlanMaxBitDegree);
    if (n >= qkdp::kPlanMaxBits)
        return set_error(QKD_ERR_UNSUPPORTED, "N=%d exceeds the plan limit %d", n, qkdp::kPlanMaxBits - 1);
    if (m > qkdp::kPlanMaxChecks)
        return set_error(QKD_ERR_UNSUPPORTED, "M=%d exceeds the plan limit %d", m, qkdp::kPlanMaxChecks);

    c->device = device;
    c->n = n;
    c->m = m;
    c->e = e;
    c->max_dc = max_dc;
    c->min_dc = max_dc;
    for (int32_t j = 0; j < m; ++j) c->min_dc = std::min(c->min_dc, cptr[j + 1] - cptr[j]);
    c->max_dv = max_dv;
    c->min_dv = *std::min_element(bdeg.begin(), bdeg.end());
    c->check_ptr.assign(cptr, cptr + m + 1);
    c->check_idx.assign(cidx, cidx + e);
    // bit side: iterate checks ascending -> each bit row ascending
    c->bit_ptr.assign(n + 1, 0);
    for (int32_t i = 0; i < n; ++i) c->bit_ptr[i + 1] = c->bit_ptr[i] + bdeg[i];
    c->bit_idx.assign(e, 0);
    std::vector<int32_t> fill(c->bit_ptr.begin(), c->bit_ptr.end() - 1);
    c->n_pad = round_up(n + 1, 64);   // column n: dummy target of idle plan lanes
    c->m_pad = round_up(m, 64);
    std::vector<int32_t> chk_bits((size_t)max_dc * c->m_pad, -1);
    std::vector<uint8_t> chk_deg(m, 0);
    std::vector<int32_t> bit_chk((size_t)max_dv * c->n_pad, -1);
    std::vector<uint8_t> bit_pos((size_t)max_dv * c->n_pad, 0);
    std::vector<uint8_t> bit_deg(n, 0);
    std::vector<int32_t> krow(e, 0);
    for (int32_t j = 0; j < m; ++j) {
        chk_deg[j] = (uint8_t)(cptr[j + 1] - cptr[j]);
        for (int32_t k = cptr[j]; k < cptr[j + 1]; ++k) {
            const int32_t slot = k - cptr[j];
            const int32_t b = cidx[k];
            chk_bits[(size_t)slot * c->m_pad + j] = b;
            const int32_t bk = fill[b] - c->bit_ptr[b];
            c->bit_idx[fill[b]++] = j;
            bit_chk[(size_t)bk * c->n_pad + b] = j;
            bit_pos[(size_t)bk * c->n_pad + b] = (uint8_t)slot;
            krow[k] = bk;
        }
    }
    qkdp::WavePlan plan;
    if (!qkdp::build_wave_plan(n, m, cptr, cidx, krow.data(), plan))
        return set_error(QKD_ERR_UNSUPPORTED, "check degree outside [1, %d]", qkdp::kPlanMaxDegree);
    c->n_tasks = plan.n_tasks;
    // degree patterns of the bits: the ascending checks' degrees
    std::vector<uint16_t> bit_pat(n, 0);
    c->n_pat = 0;
    c->pat_deg.clear();
    if (max_dv <= kTab2MaxDv) {
        std::map<std::vector<uint8_t>, int> ids;
        for (int32_t i = 0; i < n; ++i) {
            std::vector<uint8_t> key(max_dv, 0);
            for (int32_t k = c->bit_ptr[i]; k < c->bit_ptr[i + 1]; ++k) {
                const int32_t j = c->bit_idx[k];
                key[k - c->bit_ptr[i]] = (uint8_t)(cptr[j + 1] - cptr[j]);
            }
            auto it = ids.find(key);
            if (it == ids.end()) {
                it = ids.emplace(key, (int)ids.size()).first;
                c->pat_deg.insert(c->pat_deg.end(), key.begin(), key.end());
            }
            bit_pat[i] = (uint16_t)it->second;
        }
        c->n_pat = (int32_t)ids.size();
        if ((size_t)c->n_pat * tab2_stride(max_dv) > (size_t)kTab2MaxEntries) {
            c->n_pat = 0;
            c->pat_deg.clear();
        }
    }
    bool reg = true;
    for (int32_t i = 0; i < n; ++i) {
        bit_deg[i] = (uint8_t)bdeg[i];
        reg = reg && bdeg[i] == bdeg[0];
    }
    for (int32_t j = 0; j < m; ++j) reg = reg && chk_deg[j] == chk_deg[0];
    c->is_regular = reg ? 1 : 0;

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_error(QKD_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev)
        return set_error(QKD_ERR_INVALID_ARG, "device %d out of range (%d devices)", device, ndev);
    DeviceGuard g(device);
    QKD_HIP(hipDeviceGetAttribute(&c->cu_count, hipDeviceAttributeMultiprocessorCount, device));
    QKD_HIP(hipMalloc(&c->d_chk_bits, chk_bits.size() * sizeof(int32_t)));
    QKD_HIP(hipMalloc(&c->d_chk_deg, chk_deg.size()));
    QKD_HIP(hipMalloc(&c->d_bit_chk, bit_chk.size() * sizeof(int32_t)));
    QKD_HIP(hipMalloc(&c->d_bit_deg, bit_deg.size()));
    QKD_HIP(hipMemcpy(c->d_chk_bits, chk_bits.data(), chk_bits.size() * sizeof(int32_t),
                      hipMemcpyHostToDevice));
    QKD_HIP(hipMemcpy(c->d_chk_deg, chk_deg.data(), chk_deg.size(), hipMemcpyHostToDevice));
    {
        // odd-degree checks as syndrome words (qkd_decode.h decode_m_words)
        std::vector<uint32_t> odd((size_t)((m + 63) / 64) * 2, 0u);
        for (int32_t j = 0; j < m; ++j)
            if (chk_deg[j] & 1u) odd[j >> 5] |= 1u << (j & 31);
        QKD_HIP(hipMalloc(&c->d_chk_odd, odd.size() * sizeof(uint32_t)));
        QKD_HIP(hipMemcpy(c->d_chk_odd, odd.data(), odd.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    QKD_HIP(hipMalloc(&c->d_bit_pos, bit_pos.size()));
    QKD_HIP(hipMemcpy(c->d_bit_pos, bit_pos.data(), bit_pos.size(), hipMemcpyHostToDevice));
    QKD_HIP(hipMemcpy(c->d_bit_chk, bit_chk.data(), bit_chk.size() * sizeof(int32_t),
                      hipMemcpyHostToDevice));
    QKD_HIP(hipMemcpy(c->d_bit_deg, bit_deg.data(), bit_deg.size(), hipMemcpyHostToDevice));
    if (c->n_pat > 0) {
        QKD_HIP(hipMalloc(&c->d_bit_pat, bit_pat.size() * sizeof(uint16_t)));
        QKD_HIP(hipMalloc(&c->d_pat_deg, c->pat_deg.size()));
        QKD_HIP(hipMemcpy(c->d_bit_pat, bit_pat.data(), bit_pat.size() * sizeof(uint16_t),
                          hipMemcpyHostToDevice));
        QKD_HIP(hipMemcpy(c->d_pat_deg, c->pat_deg.data(), c->pat_deg.size(), hipMemcpyHostToDevice));
    }
    // The split kernels' data (decode_split.hip, decode_ilv.hip), only for
    // codes they take (N <= kMaxBitsSplitLong, M <= kMaxChecksSplit; past
    // kMaxBitsSplit only the frame-interleaved decoder and its exact hand-off
    // kernel; the launcher checks the same): larger codes run the classic
    // kernel on the original order, so the internal bit order (its bank pass
    // searches up to 200k moves) and the internal-order arrays are neither
    // computed nor uploaded for them.
    const bool split = n <= kMaxBitsSplitLong && m <= kMaxChecksSplit;
    std::vector<int32_t> perm(n), inv(n, -1);
    if (split) {
    // the split kernels' internal bit order (internal_bit_order)
    const DbgOpt bit_order = debug_option(nullptr, "QKD_BIT_ORDER");
    internal_bit_order(n, c->n_pad, bdeg, plan, perm, inv, bit_order ? bit_order.c_str() : nullptr);
    // the per-bit arrays in that order (the split kernels' DeviceCode view)
    std::vector<int32_t> bit_chk_s(bit_chk.size(), -1);
    std::vector<uint8_t> bit_deg_s(n, 0);
    for (int32_t q = 0; q < n; ++q) {
        const int32_t b = perm[q];
        bit_deg_s[q] = bit_deg[b];
        for (int32_t k = 0; k < max_dv; ++k)
            bit_chk_s[(size_t)k * c->n_pad + q] = bit_chk[(size_t)k * c->n_pad + b];
    }
    QKD_HIP(hipMalloc(&c->d_perm, (size_t)n * sizeof(int32_t)));
    QKD_HIP(hipMemcpy(c->d_perm, perm.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice));
    QKD_HIP(hipMalloc(&c->d_inv, (size_t)n * sizeof(int32_t)));
    QKD_HIP(hipMemcpy(c->d_inv, inv.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice));
    // frame_syn_sliced_kernel's check rows (N < 65535, check degree <= 16):
    // each check's bits as one or two 16-byte rows of uint16 (0xffff past
    // the row), one load per row
    if (n < 65535 && max_dc <= 16) {
        const int32_t rs = max_dc <= 8 ? 8 : 16;
        std::vector<uint16_t> rows((size_t)m * rs, 0xffff);
        for (int32_t j = 0; j < m; ++j)
            for (int32_t k = 0; k < chk_deg[j]; ++k) rows[(size_t)j * rs + k] = (uint16_t)chk_bits[(size_t)k * c->m_pad + j];
        QKD_HIP(hipMalloc(&c->d_chk_rows16, rows.size() * sizeof(uint16_t)));
        QKD_HIP(hipMemcpy(c->d_chk_rows16, rows.data(), rows.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
        c->chk_rs = rs;
    }
    QKD_HIP(hipMalloc(&c->d_bit_chk_s, bit_chk_s.size() * sizeof(int32_t)));
    QKD_HIP(hipMemcpy(c->d_bit_chk_s, bit_chk_s.data(), bit_chk_s.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    QKD_HIP(hipMalloc(&c->d_bit_deg_s, bit_deg_s.size()));
    QKD_HIP(hipMemcpy(c->d_bit_deg_s, bit_deg_s.data(), bit_deg_s.size(), hipMemcpyHostToDevice));
    if (c->n_pat > 0) {
        // (padded past the last whole load batch of the bit phases: they load
        // every round of a batch unconditionally, decode_split.hip)
        std::vector<uint16_t> bit_pat_s((size_t)round_up(n, kDecodeBlock) + kBitPadRounds * kDecodeBlock, 0);
        for (int32_t q = 0; q < n; ++q) bit_pat_s[q] = bit_pat[perm[q]];
        QKD_HIP(hipMalloc(&c->d_bit_pat_s, bit_pat_s.size() * sizeof(uint16_t)));
        QKD_HIP(hipMemcpy(c->d_bit_pat_s, bit_pat_s.data(), bit_pat_s.size() * sizeof(uint16_t),
                          hipMemcpyHostToDevice));
    }
    // packed per-bit words for the speculative bit phases (qkd_internal.h),
    // split kernels only: in the internal order
    bool packable = m <= 65536 && max_dv <= 3;
    for (int32_t j = 0; j < m && packable; ++j) packable = chk_deg[j] >= 1 && chk_deg[j] <= 16;
    // (both padded with zeros to whole kDecodeBlock rounds and kBitPadRounds
    // more: the bit phases load whole batches of rounds unconditionally,
    // decode_split.hip spec_bit_phase / sp32_bit_phase)
    const size_t rounds_pad = std::max((size_t)c->n_pad, (size_t)round_up(n, kDecodeBlock)) +
                              (size_t)kBitPadRounds * kDecodeBlock;
    if (packable) {
        std::vector<uint64_t> code(rounds_pad, 0);
        for (int32_t q = 0; q < n; ++q) {
            const int32_t i = perm[q];
            uint64_t w = (uint64_t)bdeg[i] << 48;
            for (int32_t k = 0; k < bdeg[i]; ++k) {
                const int32_t j = bit_chk[(size_t)k * c->n_pad + i];
                w |= (uint64_t)j << (16 * k);
                w |= (uint64_t)(chk_deg[j] - 1) << (50 + 4 * k);
            }
            code[q] = w;
        }
        QKD_HIP(hipMalloc(&c->d_bit_code, code.size() * sizeof(uint64_t)));
        QKD_HIP(hipMemcpy(c->d_bit_code, code.data(), code.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
        // the frame-interleaved decoder's check rows (decode_ilv.hip): each
        // edge's message line, row * n_pad + internal bit, in the check's order
        const int32_t rs = max_dc <= 8 ? 8 : 16;
        std::vector<uint32_t> lines((size_t)m * rs, 0xffffffffu);
        for (int32_t j = 0; j < m; ++j)
            for (int32_t k = cptr[j]; k < cptr[j + 1]; ++k)
                lines[(size_t)j * rs + (k - cptr[j])] = (uint32_t)krow[k] * (uint32_t)c->n_pad + (uint32_t)inv[cidx[k]];
        QKD_HIP(hipMalloc(&c->d_ilv_slots, lines.size() * sizeof(uint32_t)));
        QKD_HIP(hipMemcpy(c->d_ilv_slots, lines.data(), lines.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        c->ilv_rs = rs;
    }
    }   // split
    std::vector<uint2> plan2(plan.word.size());
    for (size_t k = 0; k < plan.word.size(); ++k) plan2[k] = make_uint2(plan.word[k], plan.seg[k]);
    QKD_HIP(hipMalloc(&c->d_plan, plan2.size() * sizeof(uint2)));
    QKD_HIP(hipMemcpy(c->d_plan, plan2.data(), plan2.size() * sizeof(uint2), hipMemcpyHostToDevice));
    if (split) {
        // the same plan slot-addressed for the split kernels (row * n_pad +
        // internal bit; idle lanes: the dummy column n's slot)
        for (size_t k = 0; k < plan.word.size(); ++k) {
            const uint32_t b = plan.word[k] & qkdp::kPlanBitMask;
            plan2[k].x = (plan.word[k] >> 24) * (uint32_t)c->n_pad + (b < (uint32_t)n ? (uint32_t)inv[b] : b);
        }
        QKD_HIP(hipMalloc(&c->d_plan_slot, plan2.size() * sizeof(uint2)));
        QKD_HIP(hipMemcpy(c->d_plan_slot, plan2.data(), plan2.size() * sizeof(uint2), hipMemcpyHostToDevice));
        c->plan_slot_host = std::move(plan2);
    }
    // Key-generation jump-ahead: chunk = draws per lane, a multiple of 64 so
    // every lane's Alice bits fill whole words.
    const uint64_t draws = qkdr::trial_draws((uint32_t)n);
    const uint64_t per_lane = (draws + kKeygenLanes - 1) / kKeygenLanes;
    c->keygen_chunk = (uint32_t)((per_lane + 63) / 64 * 64);
    std::vector<uint64_t> jump((size_t)kKeygenLevels * 256 * 4);
    qkdr::xoshiro_jump_matrices(c->keygen_chunk, kKeygenLevels, jump.data());
    QKD_HIP(hipMalloc(&c->d_jump, jump.size() * sizeof(uint64_t)));
    QKD_HIP(hipMemcpy(c->d_jump, jump.data(), jump.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    // the same jumps as polynomials, one per lane: x^(l * chunk) mod P (the
    // default form, qkd_rng.h jump_poly_apply)
    std::vector<uint64_t> jp((size_t)kKeygenLanes * 4);
    if (!qkdr::xoshiro_jump_polys(c->keygen_chunk, kKeygenLanes, jp.data()))
        return set_error(QKD_ERR_DEVICE, "xoshiro256 characteristic polynomial: unexpected degree");
    QKD_HIP(hipMalloc(&c->d_jpoly, jp.size() * sizeof(uint64_t)));
    QKD_HIP(hipMemcpy(c->d_jpoly, jp.data(), jp.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    // the two-wave generator's starts (keygen_split_kernel): Alice's bits in
    // kKgSplitLanes chunks of kg_cb, the shuffle draws (from draw N) in
    // kKgSplitLanes chunks of kg_cs
    {
        uint64_t P[4];
        if (!qkdr::xoshiro_charpoly(P))
            return set_error(QKD_ERR_DEVICE, "xoshiro256 characteristic polynomial: unexpected degree");
        const uint32_t kl = kKgSplitLanes;
        // (a multiple of 32: a lane's chunk of Alice's bits is whole 32-bit
        // words, written by that lane alone, keygen_split_kernel)
        c->kg_cb = (uint32_t)(((n + kl - 1) / kl + 31) / 32 * 32);
        c->kg_cs = (uint32_t)((draws - (uint64_t)n + kl - 1) / kl);
        std::vector<uint64_t> jp2((size_t)2 * kl * 4);
        for (uint32_t l = 0; l < kl; ++l) {
            qkdr::poly_x_pow((uint64_t)l * c->kg_cb, P, &jp2[(size_t)l * 4]);
            qkdr::poly_x_pow((uint64_t)n + (uint64_t)l * c->kg_cs, P, &jp2[(size_t)(kl + l) * 4]);
        }
        QKD_HIP(hipMalloc(&c->d_jpoly2, jp2.size() * sizeof(uint64_t)));
        QKD_HIP(hipMemcpy(c->d_jpoly2, jp2.data(), jp2.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    }
    return QKD_OK;
}

static qkd_code* make_code(int32_t n, int32_t m, const int32_t* cptr, const int32_t* cidx,
                           int device, qkd_status* status) {
    qkd_code* c = new (std::nothrow) qkd_code();
    qkd_status s = c ? build_code(c, n, m, cptr, cidx, device)
                     : set_error(QKD_ERR_OUT_OF_MEMORY, "out of host memory");
    if (s != QKD_OK) {
        free_device(c);
        delete c;
        c = nullptr;
    }
    if (status) *status = s;
    return c;
}

// ---- readers ---------------------------------------------------------------

// istringstream >> int semantics: integers up to the first non-integer token.
static void parse_ints(const std::string& line, std::vector<long>& out) {
    out.clear();
    const char* s = line.c_str();
    for (;;) {
        while (*s == ' ' || *s == '\t' || *s == '\r' || *s == '\v' || *s == '\f' || *s == '\n') s++;
        if (!*s) break;
        char* end = nullptr;
        errno = 0;
        long v = strtol(s, &end, 10);
        if (end == s || errno == ERANGE || v > INT32_MAX || v < INT32_MIN) break;
        out.push_back(v);
        s = end;
    }
}

static bool read_lines(const char* path, std::vector<std::vector<long>>& rows) {
    std::ifstream f(path);
    if (!f.is_open()) return false;
    std::string line;
    std::vector<long> v;
    while (std::getline(f, line)) {
        parse_ints(line, v);
        rows.push_back(v);
    }
    return true;
}

// read_sparse_alist_matrix (reference array_and_matrix_operations.cpp:109-292)
// sort_rows (QKD_READ_SORT_ROWS): each line's entries are sorted first, so a
// file whose rows are not ascending is read as the matrix it describes instead
// of being rejected (the reference would silently pair messages with the
// wrong edges).
static qkd_status parse_alist(const char* path, int32_t& n, int32_t& m, std::vector<int32_t>& cptr,
                              std::vector<int32_t>& cidx, bool sort_rows) {
    std::vector<std::vector<long>> v;
    if (!path || !read_lines(path, v))
        return set_error(QKD_ERR_IO, "Failed to open file: %s", path ? path : "(null)");
    if (v.empty()) return set_error(QKD_ERR_IO, "File is empty or cannot be read properly: %s", path);
    if (v.size() < 4) return set_error(QKD_ERR_IO, "Insufficient data in the file: %s", path);
    if (v[0].size() != 2 || v[1].size() != 2)
        return set_error(QKD_ERR_IO, "File format does not match the alist format: %s", path);
    const long cols = v[0][0], rows = v[0][1];
    const size_t nb = v[2].size(), nc = v[3].size();
    if (v.size() < 4 + nb + nc) return set_error(QKD_ERR_IO, "Insufficient data in the file: %s", path);
    if (cols != (long)nb)
        return set_error(QKD_ERR_IO, "Number of columns '%ld' is not the same as the length of the third line '%zu'. File: %s", cols, nb, path);
    if (rows != (long)nc)
        return set_error(QKD_ERR_IO, "Number of rows '%ld' is not the same as the length of the fourth line '%zu'. File: %s", rows, nc, path);
    for (size_t i = 0; i < nb + nc; ++i) {
        const auto& L = v[4 + i];
        const long w = i < nb ? v[2][i] : v[3][i - nb];
        long nz = 0;
        for (long x : L) nz += (x != 0);
        if (nz != w || w < 0 || (size_t)w > L.size())
            return set_error(QKD_ERR_IO, "Number of non-zero elements '%ld' in the line '%zu' does not match the weight '%ld'. File: %s", nz, 5 + i, w, path);
    }
    n = (int32_t)cols;
    m = (int32_t)rows;
    // check_nodes rows (the first weight entries of each check line, 1-based)
    cptr.assign(m + 1, 0);
    cidx.clear();
    for (int32_t j = 0; j < m; ++j) {
        const auto& L = v[4 + nb + j];
        for (long k = 0; k < v[3][j]; ++k) cidx.push_back((int32_t)(L[k] - 1));
        if (sort_rows) std::sort(cidx.begin() + cptr[j], cidx.end());
        cptr[j + 1] = (int32_t)cidx.size();
    }
    // bit_nodes rows must describe the same edge set (the reference reads
    // both and would route messages inconsistently if they disagree)
    std::vector<std::vector<int32_t>> from_checks(n);
    for (int32_t j = 0; j < m; ++j)
        for (int32_t k = cptr[j]; k < cptr[j + 1]; ++k) {
            const int32_t b = cidx[k];
            if (b < 0 || b >= n)
                return set_error(QKD_ERR_BAD_CODE, "check %d lists bit %d outside [1,%d]. File: %s", j + 1, b + 1, n, path);
            from_checks[b].push_back(j);
        }
    for (int32_t i = 0; i < n; ++i) {
        const auto& L = v[4 + i];
        std::vector<int32_t> row;
        for (long k = 0; k < v[2][i]; ++k) row.push_back((int32_t)(L[k] - 1));
        if (sort_rows) std::sort(row.begin(), row.end());
        if (row != from_checks[i]) {
            std::vector<int32_t> s = row;
            std::sort(s.begin(), s.end());
            if (s == from_checks[i])
                return set_error(QKD_ERR_UNSORTED, "bit %d: check list not ascending. File: %s", i + 1, path);
            return set_error(QKD_ERR_BAD_CODE, "bit %d: check list disagrees with the check rows. File: %s", i + 1, path);
        }
    }
    return QKD_OK;
}

// read_dense_matrix (reference array_and_matrix_operations.cpp:295-421)
static qkd_status parse_dense(const char* path, int32_t& n, int32_t& m, std::vector<int32_t>& cptr,
                              std::vector<int32_t>& cidx) {
    std::vector<std::vector<long>> v;
    if (!path || !read_lines(path, v))
        return set_error(QKD_ERR_IO, "Failed to open file: %s", path ? path : "(null)");
    if (v.empty()) return set_error(QKD_ERR_IO, "File is empty or cannot be read properly: %s", path);
    for (const auto& r : v)
        for (long x : r)
            if (x != 0 && x != 1)
                return set_error(QKD_ERR_IO, "Parity check matrix can only take values 0 or 1. File: %s", path);
    for (const auto& r : v)
        if (r.size() != v[0].size())
            return set_error(QKD_ERR_IO, "Different lengths of rows in a matrix. File: %s", path);
    n = (int32_t)v[0].size();
    m = (int32_t)v.size();
    for (int32_t i = 0; i < n; ++i) {
        long w = 0;
        for (int32_t j = 0; j < m; ++j) w += v[j][i];
        if (w <= 0)
            return set_error(QKD_ERR_IO, "Column '%d' weight cannot be equal to or less than zero. File: %s", i + 1, path);
    }
    cptr.assign(m + 1, 0);
    cidx.clear();
    for (int32_t j = 0; j < m; ++j) {
        for (int32_t i = 0; i < n; ++i)
            if (v[j][i]) cidx.push_back(i);
        if (cidx.size() == (size_t)cptr[j])
            return set_error(QKD_ERR_IO, "Row '%d' weight cannot be equal to or less than zero. File: %s", j + 1, path);
        cptr[j + 1] = (int32_t)cidx.size();
    }
    return QKD_OK;
}

}  // namespace qkd

using namespace qkd;

extern "C" {

int qkd_abi_version(void) { return QKD_LDPC_ABI_VERSION; }

const char* qkd_last_error(void) { return g_last_error.c_str(); }

const char* qkd_status_string(qkd_status s) {
    switch (s) {
        case QKD_OK: return "ok";
        case QKD_ERR_INVALID_ARG: return "invalid argument";
        case QKD_ERR_BAD_CODE: return "malformed parity-check matrix";
        case QKD_ERR_UNSORTED: return "adjacency row not ascending";
        case QKD_ERR_QBER_TOO_SMALL: return "key size too small for QBER";
        case QKD_ERR_DEVICE: return "HIP device error";
        case QKD_ERR_OUT_OF_MEMORY: return "out of memory";
        case QKD_ERR_IO: return "matrix file error";
        case QKD_ERR_UNSUPPORTED: return "unsupported code shape";
    }
    return "unknown status";
}

int qkd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

qkd_code* qkd_code_create(int32_t n_bits, int32_t n_checks, const int32_t* check_ptr,
                          const int32_t* check_idx, int device, qkd_status* status) {
    clear_error();
    return make_code(n_bits, n_checks, check_ptr, check_idx, device, status);
}

qkd_code* qkd_code_from_alist(const char* path, int device, qkd_status* status) {
    return qkd_code_from_alist_ex(path, device, 0, status);
}

qkd_code* qkd_code_from_alist_ex(const char* path, int device, uint32_t read_flags, qkd_status* status) {
    clear_error();
    if (read_flags & ~QKD_READ_SORT_ROWS) {
        set_error(QKD_ERR_INVALID_ARG, "unknown read flags 0x%x", read_flags);
        if (status) *status = QKD_ERR_INVALID_ARG;
        return nullptr;
    }
    int32_t n = 0, m = 0;
    std::vector<int32_t> cptr, cidx;
    qkd_status s = parse_alist(path, n, m, cptr, cidx, (read_flags & QKD_READ_SORT_ROWS) != 0);
    if (s != QKD_OK) {
        if (status) *status = s;
        return nullptr;
    }
    return make_code(n, m, cptr.data(), cidx.data(), device, status);
}

qkd_code* qkd_code_from_dense(const char* path, int device, qkd_status* status) {
    clear_error();
    int32_t n = 0, m = 0;
    std::vector<int32_t> cptr, cidx;
    qkd_status s = parse_dense(path, n, m, cptr, cidx);
    if (s != QKD_OK) {
        if (status) *status = s;
        return nullptr;
    }
    return make_code(n, m, cptr.data(), cidx.data(), device, status);
}

qkd_status qkd_debug_set_option(qkd_workspace* ws, const char* name, const char* value) {
    clear_error();
    if (!name) return set_error(QKD_ERR_INVALID_ARG, "option name is null");
    bool known = false;
    for (const char* k : kDebugOptions) known = known || !strcmp(k, name);
    if (!known) return set_error(QKD_ERR_INVALID_ARG, "unknown debug option '%s'", name);
    std::lock_guard<std::mutex> lock(g_dbg_mu);
    std::map<std::string, std::string>& m = ws ? ws->dbg : g_dbg;
    if (value) m[name] = value;
    else m.erase(name);
    return QKD_OK;
}

void qkd_code_destroy(qkd_code* code) {
    if (!code) return;
    if (code->default_ws) qkd_workspace_destroy(code->default_ws);
    free_device(code);
    delete code;
}

qkd_status qkd_code_get_info(const qkd_code* c, qkd_code_info* info) {
    if (!c || !info) return set_error(QKD_ERR_INVALID_ARG, "null argument");
    info->n_bits = c->n;
    info->n_checks = c->m;
    info->n_edges = c->e;
    info->max_bit_degree = c->max_dv;
    info->max_check_degree = c->max_dc;
    info->is_regular = c->is_regular;
    info->device = c->device;
    return QKD_OK;
}

qkd_status qkd_code_get_adjacency(const qkd_code* c, int32_t* check_ptr, int32_t* check_idx,
                                  int32_t* bit_ptr, int32_t* bit_idx) {
    if (!c) return set_error(QKD_ERR_INVALID_ARG, "null code");
    if (check_ptr) std::memcpy(check_ptr, c->check_ptr.data(), c->check_ptr.size() * 4);
    if (check_idx) std::memcpy(check_idx, c->check_idx.data(), c->check_idx.size() * 4);
    if (bit_ptr) std::memcpy(bit_ptr, c->bit_ptr.data(), c->bit_ptr.size() * 4);
    if (bit_idx) std::memcpy(bit_idx, c->bit_idx.data(), c->bit_idx.size() * 4);
    return QKD_OK;
}

qkd_status qkd_debug_bit_order(int32_t n, int32_t m, const int32_t* cptr, const int32_t* cidx, const char* mode,
                               int32_t* perm_out, uint32_t* plan_out, int32_t* n_tasks_out) {
    clear_error();
    if (!n_tasks_out) return set_error(QKD_ERR_INVALID_ARG, "bad arguments");
    // (build_code's validation first: the sizes below come from cptr)
    std::vector<int32_t> bdeg;
    int32_t max_dc = 0;
    const qkd_status vs = validate_csr(n, m, cptr, cidx, bdeg, max_dc);
    if (vs != QKD_OK) return vs;
    std::vector<int32_t> fill(n, 0), krow(cptr[m]);
    for (int32_t j = 0; j < m; ++j)
        for (int32_t k = cptr[j]; k < cptr[j + 1]; ++k) krow[k] = fill[cidx[k]]++;
    qkdp::WavePlan plan;
    if (!qkdp::build_wave_plan(n, m, cptr, cidx, krow.data(), plan))
        return set_error(QKD_ERR_UNSUPPORTED, "check degree outside [1, %d]", qkdp::kPlanMaxDegree);
    const int32_t n_pad = round_up(n + 1, 64);
    std::vector<int32_t> perm(n), inv(n, -1);
    internal_bit_order(n, n_pad, bdeg, plan, perm, inv, mode);
    if (perm_out) std::copy(perm.begin(), perm.end(), perm_out);
    if (plan_out) std::copy(plan.word.begin(), plan.word.begin() + (size_t)plan.n_tasks * 64, plan_out);
    *n_tasks_out = plan.n_tasks;
    return QKD_OK;
}

qkd_status qkd_make_seeds(uint64_t simulation_seed, size_t count, uint64_t* seeds) {
    if (count && !seeds) return set_error(QKD_ERR_INVALID_ARG, "null seeds");
    qkdr::Xoshiro256pp g;
    g.seed(simulation_seed);
    for (size_t i = 0; i < count; ++i) seeds[i] = g.next();
    return QKD_OK;
}

qkd_status qkd_qber_range(double begin, double end, double step, double* values, size_t capacity,
                          size_t* count) {
    if (!count || !(step > 0.0)) return set_error(QKD_ERR_INVALID_ARG, "bad QBER range");
    const double r = std::round((end - begin) / step);
    const size_t steps = r > 0 ? (size_t)r : 0;
    for (size_t j = 0; j < steps && j < capacity && values; ++j) values[j] = begin + (double)j * step;
    *count = steps;
    return QKD_OK;
}

}  // extern "C"

// qkd_ldpc_algorithm_amd.cpp — the reference's hot-path C++ API implemented
// on the MI355X decoder (C ABI, include/qkd_ldpc.h).
//
// Drop-in for ColdCloudd/QKD_LDPC:
//   src/qkd_ldpc_algorithm.cpp      sum_product_decoding_{regular,irregular},
//                                   QKD_LDPC_{regular,irregular}
//   src/array_and_matrix_operations.cpp:463-486
//                                   calculate_syndrome_{regular,irregular}
//   src/simulation.cpp:161-189      run_trial
//   src/simulation.cpp:192-316      QKD_LDPC_batch_simulation
// with the reference's signatures, CFG-driven parameters and exceptions
// (std::runtime_error with the reference's messages where it throws). The
// single-frame calls run one frame per call (the reference's granularity);
// QKD_LDPC_batch_simulation and qkd_amd_run_trials run whole QBER points as
// one device batch, which is the intended fast path.
//
// Code objects: the first call with an H_matrix uploads it (validated CSR +
// device layouts) and caches the handle by the matrix's row-pointer array;
// each later call checks the cached rows against the matrix's (an address can
// be reused by a different matrix after free_matrix_H). Each host thread
// gets its own HIP stream and workspaces, so the reference's thread pool may
// call these functions concurrently.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/qkd_ldpc.h"
#include "qkd_amd_extensions.hpp"
#include "qkd_reference_api.hpp"
#include "qkd_sim_stats.hpp"

namespace {

[[noreturn]] void fail(const char* what) {
    const char* e = qkd_last_error();
    throw std::runtime_error(std::string(what) + ((e && *e) ? std::string(": ") + e : std::string()));
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// The device and the decoder variant of the shim's calls: explicit
// settings (qkd_amd_extensions.hpp), never the environment. Set before the
// first call (the code cache is per device).
std::atomic<int> g_device{0};
std::atomic<uint32_t> g_variant{QKD_VARIANT_SP_F64};

int device_index() { return g_device.load(); }

// ---- code cache ------------------------------------------------------------
struct CodeKey {
    const void* rows;
    size_t n, m;
    bool operator<(const CodeKey& o) const {
        if (rows != o.rows) return rows < o.rows;
        if (n != o.n) return n < o.n;
        return m < o.m;
    }
};

// A cached code keeps the adjacency it was built from. The reference frees
// matrices and reads new ones (free_matrix_H, array_and_matrix_operations.cpp:88-94;
// simulation.cpp:108,134), so a different matrix can reappear at a reused row-pointer
// address with the same n and m: every hit re-compares the rows (O(E) int compares,
// microseconds against a device call) and a mismatch rebuilds the entry.
//
// Lifetime: the cache and every call in flight hold the code by shared_ptr, and
// each cache entry carries a generation number. Per-thread workspaces are keyed by
// that number (never by the qkd_code address, which a new code may reuse), and a
// thread drops its workspaces of superseded generations on its next call; the
// superseded code object is destroyed once the last of those references goes.
struct CodeRef {
    std::shared_ptr<qkd_code> code;
    uint64_t gen = 0;
    qkd_code* get() const { return code.get(); }
};

struct CachedCode {
    CodeRef ref;
    std::vector<int32_t> ptr, idx;
};

std::mutex g_codes_mu;
// (never destroyed: no device call runs during static destruction at exit)
std::map<CodeKey, CachedCode>& codes() {
    static auto* m = new std::map<CodeKey, CachedCode>();
    return *m;
}
uint64_t g_next_gen = 1;
// generations still in the cache (read by ThreadCtx::workspace under g_codes_mu)
std::map<uint64_t, bool>& live_gens() {
    static auto* m = new std::map<uint64_t, bool>();
    return *m;
}

// Row length the reference loops over: max weights for the regular twins
// (qkd_ldpc_algorithm.cpp:50,60), per-row weights for the irregular ones.
size_t check_row_len(const H_matrix& H, size_t j) {
    return H.is_regular || !H.check_nodes_weight ? H.max_check_nodes_weight : (size_t)H.check_nodes_weight[j];
}

bool same_rows(const H_matrix& H, const CachedCode& c) {
    for (size_t j = 0; j < H.num_check_nodes; ++j) {
        const size_t len = check_row_len(H, j);
        if ((size_t)(c.ptr[j + 1] - c.ptr[j]) != len) return false;
        if (len && std::memcmp(H.check_nodes[j], c.idx.data() + c.ptr[j], len * sizeof(int32_t)) != 0)
            return false;
    }
    return true;
}

CodeRef code_for(const H_matrix& H) {
    if (!H.check_nodes || H.num_bit_nodes == 0 || H.num_check_nodes == 0)
        throw std::runtime_error("H_matrix is empty");
    const CodeKey key{H.check_nodes, H.num_bit_nodes, H.num_check_nodes};
    std::lock_guard<std::mutex> lk(g_codes_mu);
    auto it = codes().find(key);
    if (it != codes().end()) {
        if (same_rows(H, it->second)) return it->second.ref;
        live_gens().erase(it->second.ref.gen);      // superseded: freed with its last reference
        codes().erase(it);
    }
    CachedCode cc;
    cc.ptr.assign(H.num_check_nodes + 1, 0);
    for (size_t j = 0; j < H.num_check_nodes; ++j) {
        for (size_t k = 0; k < check_row_len(H, j); ++k) cc.idx.push_back(H.check_nodes[j][k]);
        cc.ptr[j + 1] = (int32_t)cc.idx.size();
    }
    qkd_status st = QKD_OK;
    qkd_code* raw = qkd_code_create((int32_t)H.num_bit_nodes, (int32_t)H.num_check_nodes, cc.ptr.data(),
                                    cc.idx.data(), device_index(), &st);
    if (!raw) fail("qkd_code_create");
    cc.ref.code = std::shared_ptr<qkd_code>(raw, qkd_code_destroy);
    cc.ref.gen = g_next_gen++;
    live_gens()[cc.ref.gen] = true;
    CodeRef r = cc.ref;
    codes().emplace(key, std::move(cc));
    return r;
}

// ---- per-thread device context --------------------------------------------
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    T* get(size_t n) {
        if (n > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
            hip_check(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)), "hipMalloc");
            cap = n;
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

struct ThreadCtx {
    hipStream_t stream = nullptr;
    // workspaces by code generation (CodeRef), each holding its code alive
    struct WsEntry {
        std::shared_ptr<qkd_code> code;
        qkd_workspace* ws;
    };
    std::map<uint64_t, WsEntry> ws;
    DevBuf<double> llr, q;
    DevBuf<uint8_t> syn, bits, alice, bob, sp, ko;
    DevBuf<uint32_t> iters;
    DevBuf<uint64_t> seeds;
    ThreadCtx() {
        hip_check(hipSetDevice(device_index()), "hipSetDevice");
        hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~ThreadCtx() {
        for (auto& kv : ws) qkd_workspace_destroy(kv.second.ws);
        if (stream) (void)hipStreamDestroy(stream);
    }
    qkd_workspace* workspace(const CodeRef& c) {
        {
            // drop the workspaces of superseded generations (and so this
            // thread's references to their codes)
            std::lock_guard<std::mutex> lk(g_codes_mu);
            for (auto it = ws.begin(); it != ws.end();) {
                if (live_gens().count(it->first)) {
                    ++it;
                    continue;
                }
                qkd_workspace_destroy(it->second.ws);
                it = ws.erase(it);
            }
        }
        auto it = ws.find(c.gen);
        if (it != ws.end()) return it->second.ws;
        qkd_status st = QKD_OK;
        qkd_workspace* w = qkd_workspace_create(c.get(), &st);
        if (!w) fail("qkd_workspace_create");
        ws.emplace(c.gen, WsEntry{c.code, w});
        return w;
    }
    void h2d(void* d, const void* h, size_t bytes) {
        hip_check(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync");
    }
    void d2h(void* h, const void* d, size_t bytes) {
        hip_check(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync");
    }
    void sync() { hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize"); }
};

ThreadCtx& ctx() {
    thread_local std::unique_ptr<ThreadCtx> c(new ThreadCtx());
    return *c;
}

uint32_t flags_from_cfg() {
    return (CFG.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD ? QKD_FLAG_THRESHOLD : 0u) | g_variant.load();
}

// The reference's `while (curr_iteration != max_num_iterations)` runs zero
// iterations for 0; the ABI takes >= 1, so 0 is answered here.
SP_result decode_one(const double* llr, const H_matrix& H, const int* syndrome, size_t max_it, double thr,
                     int* out) {
    if (max_it == 0) return {0, false};
    const CodeRef c = code_for(H);
    ThreadCtx& t = ctx();
    const size_t n = H.num_bit_nodes, m = H.num_check_nodes;
    std::vector<uint8_t> syn_h(m), bits_h(n);
    for (size_t j = 0; j < m; ++j) syn_h[j] = syndrome[j] ? 1 : 0;
    double* d_llr = t.llr.get(n);
    uint8_t* d_syn = t.syn.get(m);
    uint8_t* d_bits = t.bits.get(n);
    uint32_t* d_it = t.iters.get(1);
    uint8_t* d_ok = t.sp.get(1);
    t.h2d(d_llr, llr, n * sizeof(double));
    t.h2d(d_syn, syn_h.data(), m);
    const uint32_t cap = (uint32_t)std::min<size_t>(max_it, 0xffffffffu);
    if (qkd_decode_batch(c.get(), t.workspace(c), d_llr, d_syn, 1, cap, thr, flags_from_cfg(), d_bits, d_it, d_ok,
                         t.stream) != QKD_OK)
        fail("qkd_decode_batch");
    uint32_t it = 0;
    uint8_t ok = 0;
    t.d2h(bits_h.data(), d_bits, n);
    t.d2h(&it, d_it, 4);
    t.d2h(&ok, d_ok, 1);
    t.sync();
    for (size_t i = 0; i < n; ++i) out[i] = bits_h[i];
    return {(size_t)it, ok != 0};
}

LDPC_result qkd_one(const int* alice, const int* bob, double qber, const H_matrix& H) {
    const CodeRef c = code_for(H);
    ThreadCtx& t = ctx();
    const size_t n = H.num_bit_nodes;
    if (CFG.SUM_PRODUCT_MAX_ITERATIONS == 0) return {{0, false}, false};
    std::vector<uint8_t> a(n), b(n);
    for (size_t i = 0; i < n; ++i) {
        a[i] = alice[i] ? 1 : 0;
        b[i] = bob[i] ? 1 : 0;
    }
    uint8_t* d_a = t.alice.get(n);
    uint8_t* d_b = t.bob.get(n);
    uint32_t* d_it = t.iters.get(1);
    uint8_t* d_sp = t.sp.get(1);
    uint8_t* d_ko = t.ko.get(1);
    t.h2d(d_a, a.data(), n);
    t.h2d(d_b, b.data(), n);
    const uint32_t cap = (uint32_t)std::min<size_t>(CFG.SUM_PRODUCT_MAX_ITERATIONS, 0xffffffffu);
    if (qkd_qkd_ldpc_batch(c.get(), t.workspace(c), d_a, d_b, 1, qber, cap, CFG.SUM_PRODUCT_MSG_LLR_THRESHOLD,
                           flags_from_cfg(), nullptr, d_it, d_sp, d_ko, t.stream) != QKD_OK)
        fail("qkd_qkd_ldpc_batch");
    uint32_t it = 0;
    uint8_t sp = 0, ko = 0;
    t.d2h(&it, d_it, 4);
    t.d2h(&sp, d_sp, 1);
    t.d2h(&ko, d_ko, 1);
    t.sync();
    return {{(size_t)it, sp != 0}, ko != 0};
}

void syndrome_one(const int* bits, const H_matrix& H, int* out) {
    const CodeRef c = code_for(H);
    ThreadCtx& t = ctx();
    const size_t n = H.num_bit_nodes, m = H.num_check_nodes;
    std::vector<uint8_t> b(n), s(m);
    for (size_t i = 0; i < n; ++i) b[i] = bits[i] & 1;
    uint8_t* d_b = t.bits.get(n);
    uint8_t* d_s = t.syn.get(m);
    t.h2d(d_b, b.data(), n);
    if (qkd_syndrome_batch(c.get(), d_b, 1, d_s, t.stream) != QKD_OK) fail("qkd_syndrome_batch");
    t.d2h(s.data(), d_s, m);
    t.sync();
    for (size_t j = 0; j < m; ++j) out[j] = s[j];
}

const char* kTooSmall = "' is too small for QBER.";

}  // namespace

// ---- extensions: batched trials ---------------------------------------------

void qkd_amd_set_device(int device) { g_device.store(device); }

void qkd_amd_set_variant(const char* name) {
    uint32_t v;
    if (!name || !*name || !std::strcmp(name, "sp_f64")) v = QKD_VARIANT_SP_F64;
    else if (!std::strcmp(name, "sp_f32")) v = QKD_VARIANT_SP_F32;
    else if (!std::strcmp(name, "minsum")) v = QKD_VARIANT_MINSUM;
    else if (!std::strcmp(name, "minsum_sc")) v = QKD_VARIANT_MINSUM | QKD_MINSUM_SELF_CORRECT | QKD_MINSUM_SCALE(0.875);
    else throw std::runtime_error(std::string("qkd_amd_set_variant: unknown decoder variant '") + name + "'");
    g_variant.store(v);
}

std::vector<trial_result> qkd_amd_run_trials(const H_matrix& matrix, double QBER, const size_t* seeds,
                                             size_t count, size_t seed_offset) {
    std::vector<trial_result> res(count);
    if (count == 0) return res;
    const CodeRef c = code_for(matrix);
    ThreadCtx& t = ctx();
    const size_t chunk = 1u << 18;
    std::vector<uint32_t> it(std::min(count, chunk));
    std::vector<uint8_t> sp(it.size()), ko(it.size());
    std::vector<double> q(it.size());
    const uint32_t cap = (uint32_t)std::min<size_t>(CFG.SUM_PRODUCT_MAX_ITERATIONS, 0xffffffffu);
    for (size_t base = 0; base < count; base += chunk) {
        const size_t f = std::min(chunk, count - base);
        uint64_t* d_seeds = t.seeds.get(f);
        uint32_t* d_it = t.iters.get(f);
        uint8_t* d_sp = t.sp.get(f);
        uint8_t* d_ko = t.ko.get(f);
        double* d_q = t.q.get(f);
        t.h2d(d_seeds, seeds + base, f * sizeof(uint64_t));
        if (cap == 0) {
            // zero iterations: nothing decodes (simulation.cpp semantics via the decoder loop)
            for (size_t k = 0; k < f; ++k) res[base + k] = {{{0, false}, false}, 0.0};
            continue;
        }
        const qkd_status s = qkd_trials_batch(c.get(), t.workspace(c), d_seeds, seed_offset, f, QBER, cap,
                                              CFG.SUM_PRODUCT_MSG_LLR_THRESHOLD, flags_from_cfg(), d_it, d_sp,
                                              d_ko, d_q, nullptr, t.stream);
        if (s == QKD_ERR_QBER_TOO_SMALL)
            throw std::runtime_error("Key size '" + std::to_string(matrix.num_bit_nodes) + kTooSmall);
        if (s != QKD_OK) fail("qkd_trials_batch");
        t.d2h(it.data(), d_it, f * 4);
        t.d2h(sp.data(), d_sp, f);
        t.d2h(ko.data(), d_ko, f);
        t.d2h(q.data(), d_q, f * sizeof(double));
        t.sync();
        for (size_t k = 0; k < f; ++k) {
            res[base + k].ldpc_res.sp_res = {(size_t)it[k], sp[k] != 0};
            res[base + k].ldpc_res.keys_match = ko[k] != 0;
            res[base + k].initial_QBER = q[k];
        }
    }
    return res;
}

// ---- the reference API ---------------------------------------------------------

SP_result sum_product_decoding_regular(const double* const bit_array_llr, const H_matrix& matrix,
                                       const int* const syndrome, const size_t& max_num_iterations,
                                       const double& msg_threshold, int* const bit_array_out) {
    return decode_one(bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out);
}

SP_result sum_product_decoding_irregular(const double* const bit_array_llr, const H_matrix& matrix,
                                         const int* const syndrome, const size_t& max_num_iterations,
                                         const double& msg_threshold, int* const bit_array_out) {
    return decode_one(bit_array_llr, matrix, syndrome, max_num_iterations, msg_threshold, bit_array_out);
}

LDPC_result QKD_LDPC_regular(const int* const alice_bit_array, const int* const bob_bit_array, const double& QBER,
                             const H_matrix& matrix) {
    return qkd_one(alice_bit_array, bob_bit_array, QBER, matrix);
}

LDPC_result QKD_LDPC_irregular(const int* const alice_bit_array, const int* const bob_bit_array,
                               const double& QBER, const H_matrix& matrix) {
    return qkd_one(alice_bit_array, bob_bit_array, QBER, matrix);
}

void calculate_syndrome_regular(const int* const bit_array, const H_matrix& matrix, int* const syndrome_out) {
    syndrome_one(bit_array, matrix, syndrome_out);
}

void calculate_syndrome_irregular(const int* const bit_array, const H_matrix& matrix, int* const syndrome_out) {
    syndrome_one(bit_array, matrix, syndrome_out);
}

trial_result run_trial(const H_matrix& matrix, const double QBER, size_t seed) {
    return qkd_amd_run_trials(matrix, QBER, &seed, 1, 0)[0];
}

// simulation.cpp:192-316 with each QBER point's TRIALS_NUMBER trials as one
// device batch (in place of the thread pool's detach_loop) and the same
// seeds, numbering and statistics, computed in the reference's order.
std::vector<sim_result> QKD_LDPC_batch_simulation(const std::vector<sim_input>& sim_in) {
    size_t sim_total = 0;
    for (const auto& s : sim_in) sim_total += s.QBER.size();
    std::vector<sim_result> out(sim_total);
    std::vector<size_t> seeds(CFG.TRIALS_NUMBER);
    static_assert(sizeof(size_t) == sizeof(uint64_t), "seeds are 64-bit");
    if (qkd_make_seeds(CFG.SIMULATION_SEED, seeds.size(), reinterpret_cast<uint64_t*>(seeds.data())) != QKD_OK)
        fail("qkd_make_seeds");
    size_t curr_sim = 0;
    for (const auto& in : sim_in) {
        const H_matrix& matrix = in.matrix;
        const std::string matrix_filename = in.matrix_path.filename().string();
        for (double QBER : in.QBER) {
            const std::vector<trial_result> tr =
                qkd_amd_run_trials(matrix, QBER, seeds.data(), seeds.size(), curr_sim);
            const qkdsim::PointStats st = qkdsim::reduce_point(
                tr.size(), CFG.SUM_PRODUCT_MAX_ITERATIONS, [&](size_t k, bool& sp, bool& ko, size_t& it) {
                    sp = tr[k].ldpc_res.sp_res.syndromes_match;
                    ko = tr[k].ldpc_res.keys_match;
                    it = tr[k].ldpc_res.sp_res.iterations_num;
                });
            sim_result& s = out[curr_sim];
            s.sim_number = curr_sim;
            s.matrix_filename = matrix_filename;
            s.is_regular = matrix.is_regular;
            s.num_bit_nodes = matrix.num_bit_nodes;
            s.num_check_nodes = matrix.num_check_nodes;
            s.initial_QBER = tr.empty() ? 0.0 : tr[0].initial_QBER;
            s.iterations_successful_sp_max = st.iterations_successful_sp_max;
            s.iterations_successful_sp_min = st.iterations_successful_sp_min;
            s.iterations_successful_sp_mean = st.iterations_successful_sp_mean;
            s.iterations_successful_sp_std_dev = st.iterations_successful_sp_std_dev;
            s.ratio_trials_successful_ldpc = st.ratio_trials_successful_ldpc;
            s.ratio_trials_successful_sp = st.ratio_trials_successful_sp;
            curr_sim++;
        }
    }
    return out;
}

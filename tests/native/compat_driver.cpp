// Test driver for the C++ compatibility shim (compat/): reads commands on
// stdin, calls the reference-signature API exactly as the reference's callers
// do (example/qkd_ldpc_example.cpp, simulation.cpp), prints results. The
// pytest side (tests/test_compat.py) compares them with the oracle.
//
//   code <n> <m>                 then m lines "<deg> <bit>..." (0-based, ascending)
//   recode                       same as code with the current n, m, but the new rows go
//                                behind the SAME check_nodes pointer array (free_matrix_H
//                                then a read that reuses the address, simulation.cpp:108,134)
//   cfg <max_it> <thr> <thr_on> <trials> <seed>
//   decode                       then a line of n LLRs and a line of m syndrome bits
//   qkd <q>                      then a line of n alice bits and a line of n bob bits
//   syndrome                     then a line of n bits
//   trial <q> <seed>
//   batch <npoints> <q>...       QKD_LDPC_batch_simulation over one matrix
//   variant <name>               qkd_amd_set_variant (the shim's decoder variant)
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../compat/qkd_amd_extensions.hpp"
#include "../../compat/qkd_reference_api.hpp"

config_data CFG;

static H_matrix make_matrix(size_t n, size_t m, const std::vector<std::vector<int>>& rows) {
    H_matrix H;
    H.num_bit_nodes = n;
    H.num_check_nodes = m;
    H.check_nodes = new int*[m];
    H.check_nodes_weight = new int[m];
    std::vector<std::vector<int>> cols(n);
    for (size_t j = 0; j < m; ++j) {
        H.check_nodes_weight[j] = (int)rows[j].size();
        H.check_nodes[j] = new int[rows[j].size()];
        for (size_t k = 0; k < rows[j].size(); ++k) {
            H.check_nodes[j][k] = rows[j][k];
            cols[rows[j][k]].push_back((int)j);
        }
        H.max_check_nodes_weight = std::max(H.max_check_nodes_weight, rows[j].size());
    }
    H.bit_nodes = new int*[n];
    H.bit_nodes_weight = new int[n];
    for (size_t i = 0; i < n; ++i) {
        H.bit_nodes_weight[i] = (int)cols[i].size();
        H.bit_nodes[i] = new int[cols[i].size()];
        for (size_t k = 0; k < cols[i].size(); ++k) H.bit_nodes[i][k] = cols[i][k];
        H.max_bit_nodes_weight = std::max(H.max_bit_nodes_weight, cols[i].size());
    }
    bool reg = true;
    for (size_t i = 0; i < n; ++i) reg = reg && (size_t)H.bit_nodes_weight[i] == H.max_bit_nodes_weight;
    for (size_t j = 0; j < m; ++j) reg = reg && (size_t)H.check_nodes_weight[j] == H.max_check_nodes_weight;
    H.is_regular = reg;
    return H;
}

template <typename T>
static std::vector<T> read_line(size_t count) {
    std::vector<T> v(count);
    for (size_t i = 0; i < count; ++i) std::cin >> v[i];
    return v;
}

int main() {
    std::ios::sync_with_stdio(false);
    H_matrix H;
    std::string cmd;
    while (std::cin >> cmd) {
        try {
            if (cmd == "code") {
                size_t n, m;
                std::cin >> n >> m;
                std::vector<std::vector<int>> rows(m);
                for (size_t j = 0; j < m; ++j) {
                    size_t d;
                    std::cin >> d;
                    rows[j] = read_line<int>(d);
                }
                H = make_matrix(n, m, rows);
                std::printf("ok code %d\n", (int)H.is_regular);
            } else if (cmd == "recode") {
                std::vector<std::vector<int>> rows(H.num_check_nodes);
                for (size_t j = 0; j < H.num_check_nodes; ++j) {
                    size_t d;
                    std::cin >> d;
                    rows[j] = read_line<int>(d);
                }
                int** keep = H.check_nodes;
                for (size_t j = 0; j < H.num_check_nodes; ++j) delete[] keep[j];
                for (size_t i = 0; i < H.num_bit_nodes; ++i) delete[] H.bit_nodes[i];
                delete[] H.bit_nodes;
                delete[] H.bit_nodes_weight;
                delete[] H.check_nodes_weight;
                H_matrix fresh = make_matrix(H.num_bit_nodes, H.num_check_nodes, rows);
                for (size_t j = 0; j < H.num_check_nodes; ++j) keep[j] = fresh.check_nodes[j];
                delete[] fresh.check_nodes;
                fresh.check_nodes = keep;
                H = fresh;
                std::printf("ok recode %d\n", (int)H.is_regular);
            } else if (cmd == "variant") {
                std::string name;
                std::cin >> name;
                qkd_amd_set_variant(name.c_str());
                std::printf("ok variant\n");
            } else if (cmd == "cfg") {
                int on;
                std::cin >> CFG.SUM_PRODUCT_MAX_ITERATIONS >> CFG.SUM_PRODUCT_MSG_LLR_THRESHOLD >> on >>
                    CFG.TRIALS_NUMBER >> CFG.SIMULATION_SEED;
                CFG.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD = on != 0;
                std::printf("ok cfg\n");
            } else if (cmd == "decode") {
                const auto llr = read_line<double>(H.num_bit_nodes);
                const auto syn = read_line<int>(H.num_check_nodes);
                std::vector<int> out(H.num_bit_nodes, 0);
                const SP_result r =
                    H.is_regular ? sum_product_decoding_regular(llr.data(), H, syn.data(), CFG.SUM_PRODUCT_MAX_ITERATIONS,
                                                                CFG.SUM_PRODUCT_MSG_LLR_THRESHOLD, out.data())
                                 : sum_product_decoding_irregular(llr.data(), H, syn.data(),
                                                                  CFG.SUM_PRODUCT_MAX_ITERATIONS,
                                                                  CFG.SUM_PRODUCT_MSG_LLR_THRESHOLD, out.data());
                std::printf("decode %zu %d", r.iterations_num, (int)r.syndromes_match);
                for (int b : out) std::printf(" %d", b);
                std::printf("\n");
            } else if (cmd == "qkd") {
                double q;
                std::cin >> q;
                const auto a = read_line<int>(H.num_bit_nodes);
                const auto b = read_line<int>(H.num_bit_nodes);
                const LDPC_result r = H.is_regular ? QKD_LDPC_regular(a.data(), b.data(), q, H)
                                                   : QKD_LDPC_irregular(a.data(), b.data(), q, H);
                std::printf("qkd %zu %d %d\n", r.sp_res.iterations_num, (int)r.sp_res.syndromes_match,
                            (int)r.keys_match);
            } else if (cmd == "syndrome") {
                const auto bits = read_line<int>(H.num_bit_nodes);
                std::vector<int> s(H.num_check_nodes);
                if (H.is_regular) calculate_syndrome_regular(bits.data(), H, s.data());
                else calculate_syndrome_irregular(bits.data(), H, s.data());
                std::printf("syndrome");
                for (int x : s) std::printf(" %d", x);
                std::printf("\n");
            } else if (cmd == "trial") {
                double q;
                size_t seed;
                std::cin >> q >> seed;
                const trial_result r = run_trial(H, q, seed);
                std::printf("trial %zu %d %d %.17g\n", r.ldpc_res.sp_res.iterations_num,
                            (int)r.ldpc_res.sp_res.syndromes_match, (int)r.ldpc_res.keys_match, r.initial_QBER);
            } else if (cmd == "batch") {
                size_t np;
                std::cin >> np;
                sim_input in;
                in.matrix_path = "code.alist";
                in.QBER = read_line<double>(np);
                in.matrix = H;
                const std::vector<sim_result> res = QKD_LDPC_batch_simulation({in});
                for (const auto& s : res)
                    std::printf("point %zu %.17g %.17g %.17g %zu %zu %.17g %.17g\n", s.sim_number, s.initial_QBER,
                                s.iterations_successful_sp_mean, s.iterations_successful_sp_std_dev,
                                s.iterations_successful_sp_min, s.iterations_successful_sp_max,
                                s.ratio_trials_successful_sp, s.ratio_trials_successful_ldpc);
            } else {
                std::printf("error unknown command %s\n", cmd.c_str());
            }
        } catch (const std::exception& e) {
            std::printf("exception %s\n", e.what());
        }
        std::fflush(stdout);
    }
    return 0;
}

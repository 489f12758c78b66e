// qkd_ldpc_sim — the reference's batch-mode program on MI355X.
//
// Does what the reference's executable does in batch mode (src/main.cpp:15-68):
// read config.json (src/config.cpp:4-115, same keys, validation and
// messages), read every matrix file of dense_matrices/ or
// alist_sparse_matrices/ (directory order, as main.cpp lists them), build each
// matrix's QBER grid from its code rate (get_rate_based_QBER_range,
// simulation.cpp:48-70), run TRIALS_NUMBER trials per QBER point with the
// reference's seeds (simulation.cpp:222-249) and write the results CSV
// (write_file, simulation.cpp:4-45: same file name, `_n` suffix, columns,
// separators and number formatting). The statistics are the reference's exact
// double arithmetic over the per-trial outcomes (qkd_sim_stats.hpp), so the CSV
// rows agree with the reference's to the printed digit.
//
// What changes: each QBER point is one device batch (qkd_trials_batch: key
// generation, decoding and comparison fused) instead of TRIALS_NUMBER
// thread-pool tasks; `threads_number` is read and validated but unused;
// --gpus N (or --devices i,j,...) splits every point's trials into contiguous
// slices, one per listed device, run concurrently and concatenated in trial
// order, so the output does not depend on the split. --dry-run prints the
// matrices and QBER grids and stops before any device work.
//
// Interactive mode (config "interactive_mode": true; main.cpp:24-27 ->
// QKD_LDPC_interactive_simulation, simulation.cpp:73-137, select_matrix_file
// :160-178): the same prompts, the file index read from stdin, and per QBER
// point the reference's lines, with every point's key pair drawn from ONE
// xoshiro256++(simulation_seed) stream (qkd_interactive_batch).
//
//   qkd_ldpc_sim [--root DIR] [--config FILE] [--matrix-dir DIR] [--results-dir DIR]
//                [--gpus N | --devices i,j,...] [--variant sp_f64|sp_f32|minsum|minsum_sc]
//                [--dry-run] [--sort-rows] [--quiet]
//
// --sort-rows reads alist files whose lines are not ascending (rejected by
// default: the reference would mis-route their messages).
// DIR defaults to the current directory and plays the reference's SOURCE_DIR:
// DIR/config.json, DIR/dense_matrices, DIR/alist_sparse_matrices, DIR/results.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../include/qkd_ldpc.h"
#include "qkd_json.hpp"
#include "qkd_sim_stats.hpp"

namespace fs = std::filesystem;

namespace {

// src/config.hpp:14-21, :23-63
struct RQberParams {
    double code_rate, QBER_begin, QBER_end, QBER_step;
};

struct Config {
    size_t THREADS_NUMBER = 0, TRIALS_NUMBER = 0, SIMULATION_SEED = 0, SUM_PRODUCT_MAX_ITERATIONS = 0;
    bool INTERACTIVE_MODE = false, USE_DENSE_MATRICES = false, TRACE_QKD_LDPC = false, TRACE_SUM_PRODUCT = false,
         TRACE_SUM_PRODUCT_LLR = false, ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD = false;
    double SUM_PRODUCT_MSG_LLR_THRESHOLD = 0;
    std::vector<RQberParams> R_QBER_PARAMETERS;
};

// get_config_data (src/config.cpp:4-115)
Config get_config_data(const fs::path& config_path) {
    if (!fs::exists(config_path)) throw std::runtime_error("Configuration file not found: " + config_path.string());
    std::ifstream f(config_path);
    if (!f.is_open()) throw std::runtime_error("Failed to open configuration file: " + config_path.string());
    std::stringstream ss;
    ss << f.rdbuf();
    const qkdjson::Value config = qkdjson::parse(ss.str());
    if (config.kind == qkdjson::Value::Null ||
        (config.kind == qkdjson::Value::Object && config.fields.empty()) ||
        (config.kind == qkdjson::Value::Array && config.items.empty()))
        throw std::runtime_error("Configuration file is empty: " + config_path.string());
    try {
        Config cfg;
        cfg.THREADS_NUMBER = config["threads_number"].as_size();
        if (cfg.THREADS_NUMBER < 1) throw std::runtime_error("Number of threads must be >= 1!");
        cfg.TRIALS_NUMBER = config["trials_number"].as_size();
        if (cfg.TRIALS_NUMBER < 1) throw std::runtime_error("Number of trials must be >= 1!");
        if (config["use_config_simulation_seed"].as_bool())
            cfg.SIMULATION_SEED = config["simulation_seed"].as_size();
        else
            cfg.SIMULATION_SEED = (size_t)time(nullptr);
        cfg.INTERACTIVE_MODE = config["interactive_mode"].as_bool();
        cfg.SUM_PRODUCT_MAX_ITERATIONS = config["sum_product_max_iterations"].as_size();
        if (cfg.SUM_PRODUCT_MAX_ITERATIONS < 1)
            throw std::runtime_error("Minimum number of sum-product iterations must be >= 1!");
        cfg.USE_DENSE_MATRICES = config["use_dense_matrices"].as_bool();
        cfg.TRACE_QKD_LDPC = config["trace_qkd_ldpc"].as_bool();
        cfg.TRACE_SUM_PRODUCT = config["trace_sum_product"].as_bool();
        cfg.TRACE_SUM_PRODUCT_LLR = config["trace_sum_product_llr"].as_bool();
        cfg.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD = config["enable_sum_product_msg_llr_threshold"].as_bool();
        if (cfg.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD) {
            cfg.SUM_PRODUCT_MSG_LLR_THRESHOLD = config["sum_product_msg_llr_threshold"].as_double();
            if (cfg.SUM_PRODUCT_MSG_LLR_THRESHOLD <= 0.)
                throw std::runtime_error("Sum-product message LLR threshold must be > 0!");
        }
        const qkdjson::Value& params = config["code_rate_QBER_parameters"];
        if (params.kind == qkdjson::Value::Array)
            for (const auto& p : params.items)
                cfg.R_QBER_PARAMETERS.push_back({p["code_rate"].as_double(), p["QBER_begin"].as_double(),
                                                 p["QBER_end"].as_double(), p["QBER_step"].as_double()});
        if (cfg.R_QBER_PARAMETERS.empty()) throw std::runtime_error("Array with code rate and QBER parameters is empty!");
        for (const auto& r : cfg.R_QBER_PARAMETERS) {
            if (r.code_rate <= 0. || r.code_rate >= 1.) throw std::runtime_error("Code rate(R) must be: 0 < R < 1!");
            if (r.QBER_begin <= 0. || r.QBER_begin >= 1. || r.QBER_end <= 0. || r.QBER_end >= 1. ||
                r.QBER_begin >= r.QBER_end)
                throw std::runtime_error(
                    "Invalid QBER begin or end parameters. QBER must be: 0 < QBER < 1, and begin must be less than end.");
            if (r.QBER_step <= 0.) throw std::runtime_error("QBER step must be > 0!");
            const double epsilon = 1e-6;
            if (r.QBER_step - epsilon > r.QBER_end - r.QBER_begin) throw std::runtime_error("QBER step is too large.");
        }
        std::sort(cfg.R_QBER_PARAMETERS.begin(), cfg.R_QBER_PARAMETERS.end(),
                  [](const RQberParams& a, const RQberParams& b) { return a.code_rate < b.code_rate; });
        return cfg;
    } catch (const std::exception&) {
        std::fprintf(stderr, "An error occurred while reading a configuration parameter.\n");
        throw;
    }
}

// get_rate_based_QBER_range (src/simulation.cpp:48-70)
std::vector<double> get_rate_based_QBER_range(double code_rate, const std::vector<RQberParams>& params) {
    std::vector<double> QBER;
    for (const auto& p : params) {
        if (code_rate <= p.code_rate) {
            const size_t steps = (size_t)round((p.QBER_end - p.QBER_begin) / p.QBER_step);
            for (size_t j = 0; j < steps; j++) QBER.push_back(p.QBER_begin + j * p.QBER_step);
            break;
        }
    }
    if (QBER.empty()) throw std::runtime_error("An error occurred when generating a QBER range based on code rate.");
    return QBER;
}

// src/simulation.hpp:29-43
struct SimResult {
    size_t sim_number = 0;
    std::string matrix_filename;
    bool is_regular = false;
    size_t num_bit_nodes = 0, num_check_nodes = 0;
    double initial_QBER = 0;
    qkdsim::PointStats st;
};

// write_file (src/simulation.cpp:4-45)
fs::path write_file(const std::vector<SimResult>& data, const fs::path& directory, const Config& cfg) {
    if (!fs::exists(directory)) fs::create_directories(directory);
    const std::string base_filename = "ldpc(trial_num=" + std::to_string(cfg.TRIALS_NUMBER) +
                                      ",max_sum_prod_iters=" + std::to_string(cfg.SUM_PRODUCT_MAX_ITERATIONS) +
                                      ",seed=" + std::to_string(cfg.SIMULATION_SEED) + ")";
    const std::string extension = ".csv";
    fs::path result_file_path = directory / (base_filename + extension);
    size_t file_count = 1;
    while (fs::exists(result_file_path)) {
        result_file_path = directory / (base_filename + "_" + std::to_string(file_count) + extension);
        file_count++;
    }
    std::fstream fout;
    fout.open(result_file_path, std::ios::out | std::ios::trunc);
    if (!fout.is_open()) throw std::runtime_error("An error occurred while writing to the file.");
    fout << "\xE2\x84\x96;MATRIX_FILENAME;TYPE;CODE_RATE;M;N;QBER;ITERATIONS_SUCCESSFUL_SP_MEAN;"
            "ITERATIONS_SUCCESSFUL_SP_STD_DEV;ITERATIONS_SUCCESSFUL_SP_MIN;ITERATIONS_SUCCESSFUL_SP_MAX;"
         << "RATIO_TRIALS_SUCCESSFUL_SP;RATIO_TRIALS_SUCCESSFUL_LDPC;FER\n";
    for (const auto& d : data) {
        fout << d.sim_number << ";" << d.matrix_filename << ";" << (d.is_regular ? "regular" : "irregular") << ";"
             << 1. - (static_cast<double>(d.num_check_nodes) / d.num_bit_nodes) << ";" << d.num_check_nodes << ";"
             << d.num_bit_nodes << ";" << d.initial_QBER << ";" << d.st.iterations_successful_sp_mean << ";"
             << d.st.iterations_successful_sp_std_dev << ";" << d.st.iterations_successful_sp_min << ";"
             << d.st.iterations_successful_sp_max << ";" << d.st.ratio_trials_successful_sp << ";"
             << d.st.ratio_trials_successful_ldpc << ";" << 1. - d.st.ratio_trials_successful_ldpc << "\n";
    }
    fout.close();
    return result_file_path;
}

// Dimensions of a matrix file without building it (for --dry-run): the alist
// header "N M" (read_sparse_alist_matrix, array_and_matrix_operations.cpp:109)
// or the dense file's row count and row length (read_dense_matrix).
void read_dims(const fs::path& path, bool dense, size_t& n, size_t& m) {
    std::ifstream f(path);
    if (!f.is_open()) throw std::runtime_error("Failed to open matrix file: " + path.string());
    if (!dense) {
        if (!(f >> n >> m)) throw std::runtime_error("Malformed alist header: " + path.string());
        return;
    }
    std::string line;
    n = m = 0;
    while (std::getline(f, line)) {
        size_t cols = 0;
        for (char ch : line)
            if (ch == '0' || ch == '1') ++cols;
        if (cols == 0) continue;
        n = cols;
        ++m;
    }
    if (m == 0) throw std::runtime_error("Empty dense matrix file: " + path.string());
}

[[noreturn]] void fail(const std::string& what) {
    const char* e = qkd_last_error();
    throw std::runtime_error((e && *e) ? std::string(e) : what);
}

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// One device's share of a QBER point: code, workspace, stream, buffers.
struct Device {
    int index = 0;
    qkd_code* code = nullptr;
    qkd_workspace* ws = nullptr;
    hipStream_t stream = nullptr;
    uint64_t* seeds = nullptr;
    uint32_t* iters = nullptr;
    uint8_t *sp = nullptr, *ko = nullptr;
    double* q = nullptr;
    qkd_counters* counters = nullptr;
    size_t cap = 0;

    void reserve(size_t n) {
        if (n <= cap) return;
        release_buffers();
        hip_ok(hipSetDevice(index), "hipSetDevice");
        hip_ok(hipMalloc(&seeds, n * 8), "hipMalloc");
        hip_ok(hipMalloc(&iters, n * 4), "hipMalloc");
        hip_ok(hipMalloc(&sp, n), "hipMalloc");
        hip_ok(hipMalloc(&ko, n), "hipMalloc");
        hip_ok(hipMalloc(&q, n * 8), "hipMalloc");
        if (!counters) hip_ok(hipMalloc(&counters, sizeof(qkd_counters)), "hipMalloc");
        cap = n;
    }
    void release_buffers() {
        for (void* p : {(void*)seeds, (void*)iters, (void*)sp, (void*)ko, (void*)q})
            if (p) (void)hipFree(p);
        seeds = nullptr;
        iters = nullptr;
        sp = ko = nullptr;
        q = nullptr;
        cap = 0;
    }
    void release() {
        release_buffers();
        if (counters) (void)hipFree(counters);
        counters = nullptr;
        if (ws) qkd_workspace_destroy(ws);
        if (code) qkd_code_destroy(code);
        if (stream) (void)hipStreamDestroy(stream);
        ws = nullptr;
        code = nullptr;
        stream = nullptr;
    }
};

struct Args {
    fs::path root = ".", config, matrix_dir, results_dir;
    std::vector<int> devices{0};
    uint32_t variant = QKD_VARIANT_SP_F64;
    bool quiet = false, dry_run = false, sort_rows = false;
};

Args parse_args(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        const std::string k = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) throw std::runtime_error("missing value after " + k);
            return argv[++i];
        };
        if (k == "--root") a.root = next();
        else if (k == "--config") a.config = next();
        else if (k == "--matrix-dir") a.matrix_dir = next();
        else if (k == "--results-dir") a.results_dir = next();
        else if (k == "--gpus") {
            const int g = std::atoi(next().c_str());
            if (g < 1) throw std::runtime_error("--gpus must be >= 1");
            a.devices.clear();
            for (int d = 0; d < g; ++d) a.devices.push_back(d);
        } else if (k == "--devices") {
            a.devices.clear();
            std::stringstream ss(next());
            std::string tok;
            while (std::getline(ss, tok, ','))
                if (!tok.empty()) a.devices.push_back(std::atoi(tok.c_str()));
            if (a.devices.empty()) throw std::runtime_error("--devices needs at least one index");
        } else if (k == "--quiet") a.quiet = true;
        else if (k == "--dry-run") a.dry_run = true;
        else if (k == "--sort-rows") a.sort_rows = true;
        else if (k == "--variant") {
            const std::string v = next();
            if (v == "sp_f64") a.variant = QKD_VARIANT_SP_F64;
            else if (v == "sp_f32") a.variant = QKD_VARIANT_SP_F32;
            else if (v == "minsum") a.variant = QKD_VARIANT_MINSUM;
            // self-corrected min-sum at its best scale
            else if (v == "minsum_sc") a.variant = QKD_VARIANT_MINSUM | QKD_MINSUM_SELF_CORRECT | QKD_MINSUM_SCALE(0.875);
            else throw std::runtime_error("unknown --variant '" + v + "'");
        } else if (k == "-h" || k == "--help") {
            std::printf("usage: qkd_ldpc_sim [--root DIR] [--config FILE] [--matrix-dir DIR] [--results-dir DIR]\n"
                        "                    [--gpus N | --devices i,j,...] [--variant sp_f64|sp_f32|minsum|minsum_sc]\n"
                        "                    [--dry-run] [--sort-rows] [--quiet]\n");
            std::exit(0);
        } else {
            throw std::runtime_error("unknown argument '" + k + "'");
        }
    }
    if (a.config.empty()) a.config = a.root / "config.json";
    if (a.results_dir.empty()) a.results_dir = a.root / "results";
    return a;
}

// fmt's "{}" of a double: the shortest string that reads back to the same value
std::string shortest(double v) {
    char buf[64];
    const auto r = std::to_chars(buf, buf + sizeof buf, v);
    return std::string(buf, r.ptr);
}

// QKD_LDPC_interactive_simulation (simulation.cpp:73-137) with
// select_matrix_file (:160-178).
int run_interactive(const Args& args, const Config& cfg, const std::vector<fs::path>& paths) {
    std::printf("Choose file: \n");
    for (size_t i = 0; i < paths.size(); ++i) std::printf("%zu. %s\n", i + 1, paths[i].filename().c_str());
    std::fflush(stdout);
    int file_index = 0;
    std::cin >> file_index;
    file_index -= 1;
    if (file_index < 0 || file_index >= static_cast<int>(paths.size())) throw std::runtime_error("Wrong file number.");
    const fs::path& path = paths[file_index];
    const int device = args.devices.empty() ? 0 : args.devices[0];
    qkd_status st = QKD_OK;
    qkd_code* code = cfg.USE_DENSE_MATRICES
                         ? qkd_code_from_dense(path.c_str(), device, &st)
                         : qkd_code_from_alist_ex(path.c_str(), device, args.sort_rows ? QKD_READ_SORT_ROWS : 0u, &st);
    if (!code) fail("cannot read matrix " + path.string());
    qkd_code_info info{};
    if (qkd_code_get_info(code, &info) != QKD_OK) fail("qkd_code_get_info");
    std::printf("%s\n", info.is_regular ? "Matrix H is regular." : "Matrix H is irregular.");
    const double code_rate = 1. - (static_cast<double>(info.n_checks) / info.n_bits);
    const std::vector<double> grid = get_rate_based_QBER_range(code_rate, cfg.R_QBER_PARAMETERS);
    const size_t P = grid.size();
    std::vector<uint32_t> it(P), err(P);
    std::vector<uint8_t> sp(P), ko(P);
    std::vector<double> q(P);
    size_t done = 0;
    const uint32_t flags = (cfg.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD ? QKD_FLAG_THRESHOLD : 0u) | args.variant;
    const double thr = cfg.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD ? cfg.SUM_PRODUCT_MSG_LLR_THRESHOLD : 100.0;
    const qkd_status s = qkd_interactive_batch(code, nullptr, cfg.SIMULATION_SEED, P, grid.data(),
                                               (uint32_t)cfg.SUM_PRODUCT_MAX_ITERATIONS, thr, flags, it.data(),
                                               sp.data(), ko.data(), q.data(), err.data(), &done);
    qkd_code_destroy(code);
    for (size_t i = 0; i < done; ++i) {
        std::printf("№:%zu\n", i + 1);
        std::printf("Actual QBER: %s\n", shortest(q[i]).c_str());
        std::printf("Number of errors in a key: %u\n", err[i]);
        std::printf("Iterations performed: %u\n", it[i]);
        std::printf("%s\n\n", (ko[i] && sp[i]) ? "Error reconciliation SUCCESSFUL" : "Error reconciliation FAILED");
    }
    if (s == QKD_ERR_QBER_TOO_SMALL) {
        std::printf("№:%zu\nActual QBER: 0\n", done + 1);
        throw std::runtime_error("Key size '" + std::to_string(info.n_bits) + "' is too small for QBER.");
    }
    if (s != QKD_OK) fail("qkd_interactive_batch");
    return 0;
}

int run(int argc, char** argv) {
    const Args args = parse_args(argc, argv);
    const Config cfg = get_config_data(args.config);
    const fs::path matrix_dir = !args.matrix_dir.empty()
                                    ? args.matrix_dir
                                    : args.root / (cfg.USE_DENSE_MATRICES ? "dense_matrices" : "alist_sparse_matrices");
    if (!args.quiet && !args.dry_run) std::printf(cfg.INTERACTIVE_MODE ? "INTERACTIVE MODE\n" : "BATCH MODE\n");
    // get_file_paths_in_directory (src/utils.cpp:20-47): regular files, directory order
    if (!fs::exists(matrix_dir) || !fs::is_directory(matrix_dir)) {
        std::fprintf(stderr, "An error occurred while getting file paths in directory: %s\n", matrix_dir.c_str());
        throw std::runtime_error("Directory doesn't exist.");
    }
    std::vector<fs::path> paths;
    for (const auto& e : fs::directory_iterator(matrix_dir))
        if (fs::is_regular_file(e.path())) paths.push_back(e.path());
    if (cfg.INTERACTIVE_MODE && !args.dry_run) return run_interactive(args, cfg, paths);
    if (paths.empty()) throw std::runtime_error("Matrix folder is empty: " + matrix_dir.string());

    if (args.dry_run) {
        // the matrices as the reader sees them and their QBER grids; no device work
        for (const auto& path : paths) {
            size_t n = 0, m = 0;
            read_dims(path, cfg.USE_DENSE_MATRICES, n, m);
            const double code_rate = 1. - (static_cast<double>(m) / n);
            const std::vector<double> grid = get_rate_based_QBER_range(code_rate, cfg.R_QBER_PARAMETERS);
            std::printf("%s N=%zu M=%zu R=%.17g QBER", path.filename().c_str(), n, m, code_rate);
            for (double q : grid) std::printf(" %.17g", q);
            std::printf("\n");
        }
        return 0;
    }
    const int ndev = qkd_device_count();
    for (int d : args.devices)
        if (d < 0 || d >= ndev)
            throw std::runtime_error("device " + std::to_string(d) + " requested but " + std::to_string(ndev) +
                                     " HIP device(s) visible");
    std::vector<uint64_t> seeds(cfg.TRIALS_NUMBER);
    if (qkd_make_seeds(cfg.SIMULATION_SEED, seeds.size(), seeds.data()) != QKD_OK) fail("qkd_make_seeds");
    const uint32_t flags = (cfg.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD ? QKD_FLAG_THRESHOLD : 0u) | args.variant;
    const double thr = cfg.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD ? cfg.SUM_PRODUCT_MSG_LLR_THRESHOLD : 100.0;
    const size_t T = cfg.TRIALS_NUMBER;

    std::vector<Device> dev(args.devices.size());
    for (size_t g = 0; g < dev.size(); ++g) {
        dev[g].index = args.devices[g];
        hip_ok(hipSetDevice(dev[g].index), "hipSetDevice");
        hip_ok(hipStreamCreateWithFlags(&dev[g].stream, hipStreamNonBlocking), "hipStreamCreate");
    }
    std::vector<uint32_t> h_it(T);
    std::vector<uint8_t> h_sp(T), h_ko(T);
    std::vector<double> h_q(T);
    std::vector<SimResult> results;
    size_t curr_sim = 0;
    try {
        for (const auto& path : paths) {
            // prepare_sim_inputs (simulation.cpp:140-158): read the matrix, its QBER grid
            for (auto& d : dev) {
                qkd_status st = QKD_OK;
                d.code = cfg.USE_DENSE_MATRICES
                             ? qkd_code_from_dense(path.c_str(), d.index, &st)
                             : qkd_code_from_alist_ex(path.c_str(), d.index, args.sort_rows ? QKD_READ_SORT_ROWS : 0u, &st);
                if (!d.code) fail("cannot read matrix " + path.string());
                d.ws = qkd_workspace_create(d.code, &st);
                if (!d.ws) fail("qkd_workspace_create");
            }
            qkd_code_info info{};
            if (qkd_code_get_info(dev[0].code, &info) != QKD_OK) fail("qkd_code_get_info");
            const double code_rate = 1. - (static_cast<double>(info.n_checks) / info.n_bits);
            const std::vector<double> grid = get_rate_based_QBER_range(code_rate, cfg.R_QBER_PARAMETERS);
            for (double QBER : grid) {
                std::vector<std::string> errors(dev.size());
                std::vector<std::thread> th;
                for (size_t g = 0; g < dev.size(); ++g) {
                    th.emplace_back([&, g]() {
                        try {
                            Device& d = dev[g];
                            const size_t b = T * g / dev.size(), e = T * (g + 1) / dev.size();
                            const size_t n = e - b;
                            if (n == 0) return;
                            d.reserve(n);
                            hip_ok(hipSetDevice(d.index), "hipSetDevice");
                            hip_ok(hipMemcpyAsync(d.seeds, seeds.data() + b, n * 8, hipMemcpyHostToDevice, d.stream),
                                   "hipMemcpyAsync");
                            // frame k of point curr_sim uses seeds[k] + curr_sim (simulation.cpp:247)
                            if (qkd_trials_batch(d.code, d.ws, d.seeds, curr_sim, n, QBER,
                                                 (uint32_t)cfg.SUM_PRODUCT_MAX_ITERATIONS, thr, flags, d.iters, d.sp,
                                                 d.ko, d.q, d.counters, d.stream) != QKD_OK)
                                fail("qkd_trials_batch");
                            hip_ok(hipMemcpyAsync(h_it.data() + b, d.iters, n * 4, hipMemcpyDeviceToHost, d.stream),
                                   "hipMemcpyAsync");
                            hip_ok(hipMemcpyAsync(h_sp.data() + b, d.sp, n, hipMemcpyDeviceToHost, d.stream),
                                   "hipMemcpyAsync");
                            hip_ok(hipMemcpyAsync(h_ko.data() + b, d.ko, n, hipMemcpyDeviceToHost, d.stream),
                                   "hipMemcpyAsync");
                            hip_ok(hipMemcpyAsync(h_q.data() + b, d.q, n * 8, hipMemcpyDeviceToHost, d.stream),
                                   "hipMemcpyAsync");
                            hip_ok(hipStreamSynchronize(d.stream), "hipStreamSynchronize");
                        } catch (const std::exception& ex) {
                            errors[g] = ex.what();
                        }
                    });
                }
                for (auto& t : th) t.join();
                for (const auto& e : errors)
                    if (!e.empty()) throw std::runtime_error(e);
                SimResult r;
                r.sim_number = curr_sim;
                r.matrix_filename = path.filename().string();
                r.is_regular = info.is_regular != 0;
                r.num_bit_nodes = (size_t)info.n_bits;
                r.num_check_nodes = (size_t)info.n_checks;
                r.initial_QBER = h_q[0];
                r.st = qkdsim::reduce_point(T, cfg.SUM_PRODUCT_MAX_ITERATIONS,
                                            [&](size_t k, bool& sp, bool& ko, size_t& it) {
                                                sp = h_sp[k] != 0;
                                                ko = h_ko[k] != 0;
                                                it = h_it[k];
                                            });
                if (!args.quiet)
                    std::printf("%zu %s QBER=%g FER=%g mean_it=%g\n", curr_sim, r.matrix_filename.c_str(),
                                r.initial_QBER, 1. - r.st.ratio_trials_successful_ldpc,
                                r.st.iterations_successful_sp_mean);
                results.push_back(r);
                curr_sim++;
            }
            for (auto& d : dev) {
                qkd_workspace_destroy(d.ws);
                qkd_code_destroy(d.code);
                d.ws = nullptr;
                d.code = nullptr;
            }
        }
    } catch (...) {
        for (auto& d : dev) d.release();
        throw;
    }
    for (auto& d : dev) d.release();
    const fs::path out = write_file(results, args.results_dir, cfg);
    if (!args.quiet) std::printf("The results were written to: %s\n", out.c_str());
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        return run(argc, argv);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ERROR: %s\n", e.what());
        return EXIT_FAILURE;
    }
}

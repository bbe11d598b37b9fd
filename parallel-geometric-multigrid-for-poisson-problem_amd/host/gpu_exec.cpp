// gpu_exec.cpp — the reference's `gpu_exec` entry (3_part_parallel/main.cu:5-50) on
// MI355X: same default run (N = 33 ... 2049, 3 cycles, alpha = 3, V then W per N),
// same stdout and OUTPUT_RESULT/timings_parallel_{v,w}_cycle.txt.
//
//   gpu_exec                       # the reference's default run
//   gpu_exec --n 513,1025 --cycles 1 --alpha 3 [--ops] [--hash] [--err-vector 8193]
// --ops additionally runs the per-op timing study (plotTimeSequentialVsParallel);
// --hash prints phi's FNV-64 after every cycle run (the golden fixtures' checksum);
// --v-only runs run_v_cycle per N (no W-cycles), --warmup W adds W untimed cycles before
// the timed ones (bench.py's drop-in leg);
// --host-arrays keeps phi and f in host memory (uploaded / downloaded per cycle) instead of
// device arrays updated in place (the default, the reference's managed-memory contract);
// --err-vector N,... runs main.cu:44-47's GPU block instead of the default run
// (run_w_cycles_err_vector_iteration -> OUTPUT_RESULT/ERR_VECTOR/iteration_last_gpu.txt).
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <vector>

#include "ParallelTestRunner.hpp"

int main(int argc, char **argv)
{
    std::vector<int> N_list = {33, 65, 129, 257, 513, 1025, 2049};  // main.cu:3
    std::vector<int> N_thread_list = {16, 32};                        // main.cu:4
    int mg_max_iterations = 3;                                        // main.cu:17
    int alpha = 3;                                                    // main.cu:15
    bool ops = false, hash = false, host_arrays = false, v_only = false;
    int mixed = 0;
    int warmup = 0;
    std::vector<int> err_list;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--n") && i + 1 < argc) {
            N_list.clear();
            std::stringstream ss(argv[++i]);
            std::string tok;
            while (std::getline(ss, tok, ',')) N_list.push_back(std::atoi(tok.c_str()));
        } else if (!std::strcmp(argv[i], "--cycles") && i + 1 < argc) {
            mg_max_iterations = std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--alpha") && i + 1 < argc) {
            alpha = std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--ops")) {
            ops = true;
        } else if (!std::strcmp(argv[i], "--hash")) {
            hash = true;
        } else if (!std::strcmp(argv[i], "--host-arrays")) {
            host_arrays = true;
        } else if (!std::strcmp(argv[i], "--mixed-dphi-hf")) {
            mixed = 1;
        } else if (!std::strcmp(argv[i], "--mixed-hphi-df")) {
            mixed = 2;
        } else if (!std::strcmp(argv[i], "--v-only")) {
            v_only = true;
        } else if (!std::strcmp(argv[i], "--warmup") && i + 1 < argc) {
            warmup = std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--err-vector") && i + 1 < argc) {
            std::stringstream ss(argv[++i]);
            std::string tok;
            while (std::getline(ss, tok, ',')) err_list.push_back(std::atoi(tok.c_str()));
        } else {
            std::cerr << "usage: " << argv[0]
                      << " [--n 33,65,...] [--cycles K] [--alpha A] [--ops] [--hash]"
                         " [--host-arrays | --mixed-dphi-hf | --mixed-hphi-df] [--v-only]"
                         " [--warmup W] [--err-vector N,...]\n";
            return 2;
        }
    }
    try {
        ParallelTestRunner parallel_runner(0, mg_max_iterations, alpha);
        parallel_runner.print_hash = hash;
        parallel_runner.host_arrays = host_arrays;
        parallel_runner.mixed = mixed;
        parallel_runner.warmup_iterations = warmup;
        if (v_only) {
            for (int n : N_list) {
                parallel_runner.N = n;
                std::cout << "\n=== GPU Multigrid Solution for N = " << n << " ===\n";
                parallel_runner.run_v_cycle();
            }
            return 0;
        }
        if (!err_list.empty()) {
            parallel_runner.run_w_cycles_err_vector_iteration(err_list);
            return 0;
        }
        if (ops) parallel_runner.plotTimeSequentialVsParallel(N_list, N_thread_list);
        parallel_runner.run_all_cycles(N_list);
    } catch (const std::exception &e) {
        std::cerr << "gpu_exec: " << e.what() << "\n";
        return 1;
    }
    return 0;
}

// C++ controller tick through mpcqp::ConvexMpc (include/mpcqp/convex_mpc.hpp): reads C
// instances (x0, xref, lin, contact) from a raw little-endian file written by
// tests/test_cpp.py, runs them as one batch and prints the per-instance cost / status / iters,
// the winner and its first-step forces (%.17g).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mpcqp/convex_mpc.hpp"

int main(int argc, char **argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: mpc_tick N friction(0|1) C input.bin\n");
        return 2;
    }
    const int N = std::atoi(argv[1]), fric = std::atoi(argv[2]), C = std::atoi(argv[3]);
    mpcqp::ModelSpec spec = mpcqp::srbm_model(N, fric != 0);
    const int nx = 13, xr = (N + 1) * nx;
    std::vector<double> x0((size_t)C * nx), xref((size_t)C * xr), lin((size_t)C * 8);
    std::vector<uint64_t> contact((size_t)C);
    FILE *fp = std::fopen(argv[4], "rb");
    if (!fp) return 3;
    bool ok = std::fread(x0.data(), sizeof(double), x0.size(), fp) == x0.size() &&
              std::fread(xref.data(), sizeof(double), xref.size(), fp) == xref.size() &&
              std::fread(lin.data(), sizeof(double), lin.size(), fp) == lin.size() &&
              std::fread(contact.data(), sizeof(uint64_t), contact.size(), fp) == contact.size();
    std::fclose(fp);
    if (!ok) return 4;
    mpcqp::ConvexMpc mpc(spec);
    mpcqp::MpcChoice best = mpc.solve_batch(x0.data(), xref.data(), lin.data(), contact.data(), C);
    for (int c = 0; c < C; ++c)
        std::printf("inst %d %.17g %d %d\n", c, mpc.all_cost()[(size_t)c], best.status[(size_t)c],
                    mpc.all_iters()[(size_t)c]);
    std::printf("best %d %.17g", best.index, best.cost);
    for (int i = 0; i < 6 && best.index >= 0; ++i) std::printf(" %.17g", best.U[(size_t)i]);
    std::printf("\n");
    // the single-state form: candidate 0's state under every candidate's gait
    mpcqp::MpcChoice one = mpc.solve(x0.data(), xref.data(), lin.data(), contact.data(), C);
    std::printf("tick %d %.17g\n", one.index, one.cost);
    return 0;
}

// The multi-GPU group from a C++ controller (mpcqp::GroupMpc over mpcqp_group_*): reads S x C
// instances (x0, xref, lin, contact) from a raw little-endian file written by tests/test_cpp.py,
// solves them through the group on the listed devices (one RCCL communicator, one all-gather)
// and, on device 0 alone, through mpcqp_batch_solve_select; prints both selection records as
// hex words and whether the per-instance outputs agree bit for bit.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "mpcqp/convex_mpc.hpp"

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: group_test S C input.bin [device ...]\n");
        return 2;
    }
    const int S = std::atoi(argv[1]), C = std::atoi(argv[2]);
    std::vector<int> devices;
    for (int i = 4; i < argc; ++i) devices.push_back(std::atoi(argv[i]));
    if (devices.empty()) devices.push_back(0);
    const int N = 10, nx = 13, xr = (N + 1) * nx, nv = 60;
    const size_t B = (size_t)S * C;
    std::vector<double> x0(B * nx), xref(B * xr), lin(B * 8);
    std::vector<uint64_t> contact(B);
    FILE *fp = std::fopen(argv[3], "rb");
    if (!fp) return 3;
    bool ok = std::fread(x0.data(), sizeof(double), x0.size(), fp) == x0.size() &&
              std::fread(xref.data(), sizeof(double), xref.size(), fp) == xref.size() &&
              std::fread(lin.data(), sizeof(double), lin.size(), fp) == lin.size() &&
              std::fread(contact.data(), sizeof(uint64_t), contact.size(), fp) == contact.size();
    std::fclose(fp);
    if (!ok) return 4;
    mpcqp::ModelSpec spec = mpcqp::srbm_model(N, false);

    // the group, twice (the second tick reuses the other record buffer)
    mpcqp::GroupMpc grp(spec, devices);
    mpcqp::MpcChoice g1 = grp.solve_batch(x0.data(), xref.data(), lin.data(), contact.data(), S, C);
    mpcqp::MpcChoice g2 = grp.solve_batch(x0.data(), xref.data(), lin.data(), contact.data(), S, C);
    const std::vector<int64_t> rec = grp.record();

    // one context, device pointers, mpcqp_batch_solve_select
    mpcqp_ctx *ctx = nullptr;
    if (mpcqp_ctx_create(&spec.m, devices[0], &ctx) != MPCQP_OK) return 5;
#define CK(x) \
    do { if ((x) != hipSuccess) return 7; } while (0)
    double *dx0, *dxr, *dlin, *dU, *dc;
    uint64_t *dct;
    int *dst, *dit;
    int64_t *drec;
    CK(hipMalloc(&dx0, sizeof(double) * x0.size()));
    CK(hipMalloc(&dxr, sizeof(double) * xref.size()));
    CK(hipMalloc(&dlin, sizeof(double) * lin.size()));
    CK(hipMalloc(&dct, sizeof(uint64_t) * B));
    CK(hipMalloc(&dU, sizeof(double) * B * nv));
    CK(hipMalloc(&dc, sizeof(double) * B));
    CK(hipMalloc(&dst, sizeof(int) * B));
    CK(hipMalloc(&dit, sizeof(int) * B));
    CK(hipMalloc(&drec, sizeof(int64_t) * (1 + nv)));
    CK(hipMemcpy(dx0, x0.data(), sizeof(double) * x0.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dxr, xref.data(), sizeof(double) * xref.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dlin, lin.data(), sizeof(double) * lin.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dct, contact.data(), sizeof(uint64_t) * B, hipMemcpyHostToDevice));
    if (mpcqp_batch_solve_select(ctx, (int)B, dx0, dxr, dlin, dct, dU, dc, dst, dit, 0, drec) !=
            MPCQP_OK ||
        mpcqp_sync(ctx) != MPCQP_OK)
        return 6;
    std::vector<int64_t> rec1(1 + nv);
    std::vector<double> U1(B * nv), c1(B);
    std::vector<int> st1(B), it1(B);
    CK(hipMemcpy(rec1.data(), drec, sizeof(int64_t) * rec1.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(U1.data(), dU, sizeof(double) * U1.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(c1.data(), dc, sizeof(double) * B, hipMemcpyDeviceToHost));
    CK(hipMemcpy(st1.data(), dst, sizeof(int) * B, hipMemcpyDeviceToHost));
    CK(hipMemcpy(it1.data(), dit, sizeof(int) * B, hipMemcpyDeviceToHost));
    mpcqp_ctx_destroy(ctx);

    const bool same_out = std::memcmp(U1.data(), grp.all_U().data(), sizeof(double) * U1.size()) == 0 &&
                          std::memcmp(c1.data(), grp.all_cost().data(), sizeof(double) * B) == 0 &&
                          std::memcmp(it1.data(), grp.all_iters().data(), sizeof(int) * B) == 0 &&
                          std::memcmp(st1.data(), g2.status.data(), sizeof(int) * B) == 0;
    const bool same_rec = std::memcmp(rec.data(), rec1.data(), sizeof(int64_t) * rec1.size()) == 0;
    std::printf("group_index %d %d ctx_index %d\n", g1.index, g2.index,
                rec1[0] == INT64_MAX ? -1 : (int)(rec1[0] & 0x7fffffff));
    std::printf("group_rec");
    for (int64_t w : rec) std::printf(" %016" PRIx64, (uint64_t)w);
    std::printf("\nctx_rec");
    for (int64_t w : rec1) std::printf(" %016" PRIx64, (uint64_t)w);
    std::printf("\nsame_outputs %d same_record %d\n", same_out ? 1 : 0, same_rec ? 1 : 0);
    return same_out && same_rec ? 0 : 1;
}

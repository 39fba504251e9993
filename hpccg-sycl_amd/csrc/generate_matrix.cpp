// generate_matrix.cpp -- host-side problem generator (the drop-in input seam).
//
// Produces exactly what the reference generate_matrix() produces
// (generate_matrix.cpp:196-307 in Dart120/HPCCG-SYCL): an HPC_Sparse_Matrix
// with global column indices for one z-stacked slab, entries per row in
// (sz, sy, sx) stencil order, diagonal 27.0 / off-diagonal -1.0 (27.0 on the
// diagonal for the 7-point stencil as well), x0 = 0, b = 27 - (nnz_row - 1),
// xexact = 1, and total_nnz = 27 * total_nrow (the reference's approximation).
//
// Rows are filled in parallel (rows are independent once the per-row offsets
// are known: offsets come from an analytic per-row count), which the reference
// does serially; the resulting arrays are identical.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/HPC_Sparse_Matrix.hpp"
#include "../../include/hpccg_hip.h"

namespace {

inline int stencil_row_len(int ix, int iy, int nx, int ny, long long grow, long long nxy,
                           long long total, bool use_7pt)
{
    const int zl = grow - nxy >= 0, zh = grow + nxy < total;
    if (use_7pt) return 1 + (ix > 0) + (ix < nx - 1) + (iy > 0) + (iy < ny - 1) + zl + zh;
    const int cx = 1 + (ix > 0) + (ix < nx - 1);
    const int cy = 1 + (iy > 0) + (iy < ny - 1);
    return cx * cy * (1 + zl + zh);
}

}  // namespace

void destroyMatrix(HPC_Sparse_Matrix*& A)
{
    if (!A) return;
    hpccg_hip_dropin_release(A);  // a later matrix at this address is a new one
    delete[] A->title;
    delete[] A->nnz_in_row;
    delete[] A->list_of_vals;
    delete[] A->ptr_to_vals_in_row;
    delete[] A->list_of_inds;
    delete[] A->ptr_to_inds_in_row;
    delete[] A->ptr_to_diags;
    delete A;
    A = nullptr;
}

extern "C" int hpccg_generate_matrix(int nx, int ny, int nz, int rank, int size, int use_7pt,
                                     HPC_Sparse_Matrix** Aout, double** xout, double** bout,
                                     double** xexout)
{
    if (nx < 1 || ny < 1 || nz < 1 || size < 1 || rank < 0 || rank >= size || !Aout)
        return HPCCG_HIP_EINVAL;
    const long long n64 = (long long)nx * ny * nz;
    if (n64 * size >= (1LL << 31)) return HPCCG_HIP_EINVAL;  // int rows/cols, as the reference
    const int n = (int)n64;
    const long long nxy = (long long)nx * ny;
    const long long total = n64 * size;
    const long long start = n64 * rank;

    // per-row offsets (exclusive scan of the analytic row lengths)
    std::vector<long long> off(n + 1, 0);
    for (int i = 0; i < n; i++) {
        const int iz = (int)(i / nxy), iy = (int)((i - iz * nxy) / nx), ix = (int)(i - iz * nxy - (long long)iy * nx);
        off[i + 1] = off[i] + stencil_row_len(ix, iy, nx, ny, start + i, nxy, total, use_7pt != 0);
    }
    const long long nnz = off[n];

    auto* A = new HPC_Sparse_Matrix;
    std::memset(A, 0, sizeof *A);
    A->title = nullptr;
    A->start_row = (int)start;
    A->stop_row = (int)(start + n - 1);
    A->total_nrow = (int)total;
    A->total_nnz = 27 * total;  // generate_matrix.cpp:226 (approximation, kept)
    A->local_nrow = n;
    A->local_ncol = n;
    A->local_nnz = (int)std::min<long long>(27 * n64, 0x7fffffff);
    A->nnz_in_row = new int[n];
    A->ptr_to_vals_in_row = new double*[n];
    A->ptr_to_inds_in_row = new int*[n];
    A->ptr_to_diags = new double*[n];
    A->list_of_vals = new double[nnz > 0 ? nnz : 1];
    A->list_of_inds = new int[nnz > 0 ? nnz : 1];
    double* x = new double[n];
    double* b = new double[n];
    double* xe = new double[n];

    auto fill = [&](int lo, int hi) {
        for (int i = lo; i < hi; i++) {
            const int iz = (int)(i / nxy), iy = (int)((i - iz * nxy) / nx);
            const int ix = (int)(i - iz * nxy - (long long)iy * nx);
            const long long row = start + i;
            double* vp = A->list_of_vals + off[i];
            int* cp = A->list_of_inds + off[i];
            A->ptr_to_vals_in_row[i] = vp;
            A->ptr_to_inds_in_row[i] = cp;
            A->ptr_to_diags[i] = nullptr;
            int k = 0;
            for (int sz = -1; sz <= 1; sz++)
                for (int sy = -1; sy <= 1; sy++)
                    for (int sx = -1; sx <= 1; sx++) {
                        const long long col = row + sz * nxy + (long long)sy * nx + sx;
                        const bool inside = ix + sx >= 0 && ix + sx < nx && iy + sy >= 0 && iy + sy < ny &&
                                            col >= 0 && col < total;
                        if (!inside || (use_7pt && sz * sz + sy * sy + sx * sx > 1)) continue;
                        if (col == row) A->ptr_to_diags[i] = vp + k;
                        vp[k] = (col == row) ? 27.0 : -1.0;
                        cp[k] = (int)col;
                        k++;
                    }
            A->nnz_in_row[i] = k;
            x[i] = 0.0;
            b[i] = 27.0 - (double)(k - 1);
            xe[i] = 1.0;
        }
    };
    const int nth = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    const int chunk = (n + nth - 1) / nth;
    for (int t = 1; t < nth; t++)
        th.emplace_back(fill, std::min(n, t * chunk), std::min(n, (t + 1) * chunk));
    fill(0, std::min(n, chunk));
    for (auto& t : th) t.join();

    *Aout = A;
    if (xout) *xout = x; else delete[] x;
    if (bout) *bout = b; else delete[] b;
    if (xexout) *xexout = xe; else delete[] xe;
    return 0;
}

extern "C" void hpccg_free_problem(HPC_Sparse_Matrix* A, double* x, double* b, double* xexact)
{
    destroyMatrix(A);
    delete[] x;
    delete[] b;
    delete[] xexact;
}

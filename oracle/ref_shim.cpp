// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY (our own code, not a reference file).
//
// A thin extern "C" harness compiled TOGETHER WITH the unmodified reference
// sources under /root/reference into oracle/_ref/libhpccg_ref.so, so that the
// reference's own generate_matrix / HPC_sparsemv / ddot / waxpby / HPCCG can
// be called from Python (tests/golden/make_golden.py) to produce golden
// vectors. Nothing here re-implements reference arithmetic: every numeric
// result comes from a reference function.
//
//   ref_generate      -> generate_matrix()        generate_matrix.cpp:196
//   ref_from_csr      -> builds an HPC_Sparse_Matrix (HPC_Sparse_Matrix.hpp:54)
//                        from caller CSR, for matrices the unmodified reference
//                        generator cannot produce (7-pt, z-stacked globals)
//   ref_hpccg         -> HPCCG()                  HPCCG.cpp:312
//   ref_sparsemv      -> HPC_sparsemv()           HPC_sparsemv.cpp:68
//   ref_ddot          -> ddot()                   ddot.cpp:60
//   ref_waxpby        -> waxpby()                 waxpby.cpp:69
#include <cstring>
#include "HPC_Sparse_Matrix.hpp"
#include "generate_matrix.hpp"
#include "HPCCG.hpp"

extern "C" {

void* ref_generate(int nx, int ny, int nz, double** x, double** b, double** xexact)
{
    HPC_Sparse_Matrix* A = nullptr;
    generate_matrix(nx, ny, nz, &A, x, b, xexact);
    return A;
}

int ref_nrow(void* Av) { return static_cast<HPC_Sparse_Matrix*>(Av)->local_nrow; }

long long ref_total_nnz(void* Av) { return static_cast<HPC_Sparse_Matrix*>(Av)->total_nnz; }

// Export the matrix as CSR (row_ptr[nrow+1], cols, vals) in stored entry order.
long long ref_to_csr(void* Av, long long* row_ptr, int* cols, double* vals)
{
    HPC_Sparse_Matrix* A = static_cast<HPC_Sparse_Matrix*>(Av);
    long long k = 0;
    row_ptr[0] = 0;
    for (int i = 0; i < A->local_nrow; i++) {
        for (int j = 0; j < A->nnz_in_row[i]; j++) {
            if (cols) cols[k] = A->ptr_to_inds_in_row[i][j];
            if (vals) vals[k] = A->ptr_to_vals_in_row[i][j];
            k++;
        }
        row_ptr[i + 1] = k;
    }
    return k;
}

// Build an HPC_Sparse_Matrix (serial layout, local == global) from CSR.
void* ref_from_csr(int nrow, const long long* row_ptr, const int* cols, const double* vals)
{
    HPC_Sparse_Matrix* A = new HPC_Sparse_Matrix;
    std::memset(A, 0, sizeof(*A));
    long long nnz = row_ptr[nrow];
    A->start_row = 0;
    A->stop_row = nrow - 1;
    A->total_nrow = nrow;
    A->total_nnz = nnz;
    A->local_nrow = nrow;
    A->local_ncol = nrow;
    A->local_nnz = (int)nnz;
    A->nnz_in_row = new int[nrow];
    A->ptr_to_vals_in_row = new double*[nrow];
    A->ptr_to_inds_in_row = new int*[nrow];
    A->ptr_to_diags = new double*[nrow];
    A->list_of_vals = new double[nnz > 0 ? nnz : 1];
    A->list_of_inds = new int[nnz > 0 ? nnz : 1];
    std::memcpy(A->list_of_vals, vals, sizeof(double) * nnz);
    std::memcpy(A->list_of_inds, cols, sizeof(int) * nnz);
    for (int i = 0; i < nrow; i++) {
        A->nnz_in_row[i] = (int)(row_ptr[i + 1] - row_ptr[i]);
        A->ptr_to_vals_in_row[i] = A->list_of_vals + row_ptr[i];
        A->ptr_to_inds_in_row[i] = A->list_of_inds + row_ptr[i];
        A->ptr_to_diags[i] = nullptr;
        for (long long j = row_ptr[i]; j < row_ptr[i + 1]; j++)
            if (cols[j] == i) A->ptr_to_diags[i] = A->list_of_vals + j;
    }
    return A;
}

int ref_hpccg(void* Av, double* b, double* x, int max_iter, double tolerance,
              int* niters, double* normr, double* times)
{
    int it = 0;
    double nr = 0.0;
    int ierr = HPCCG(static_cast<HPC_Sparse_Matrix*>(Av), b, x, max_iter, tolerance, it, nr, times);
    *niters = it;
    *normr = nr;
    return ierr;
}

int ref_sparsemv(void* Av, const double* x, double* y)
{
    return HPC_sparsemv(static_cast<HPC_Sparse_Matrix*>(Av), x, y);
}

double ref_ddot(int n, const double* x, const double* y)
{
    double r = 0.0, t = 0.0;
    ddot(n, x, y, &r, t);
    return r;
}

int ref_waxpby(int n, double alpha, const double* x, double beta, const double* y, double* w)
{
    return waxpby(n, alpha, x, beta, y, w);
}

void ref_free(void* Av)
{
    HPC_Sparse_Matrix* A = static_cast<HPC_Sparse_Matrix*>(Av);
    destroyMatrix(A);
}

void ref_free_vec(double* v) { delete[] v; }

}  // extern "C"

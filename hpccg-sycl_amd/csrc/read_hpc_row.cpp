// read_hpc_row.cpp -- Mode 2 input (read_HPC_row.cpp:217-373): a linear system
// from a text file, rows block-distributed over the ranks.
//
// File format (read_HPC_row.cpp:243-345): total_nrow total_nnz, then one
// entry count per row, then per row "nnz (value column)*", then one
// "x b xexact" line per row. Rank r of P owns rows [off, off + mp) with
// chunksize = n / P, remainder = n % P, mp = chunksize + (r < remainder),
// off = r * (chunksize + 1) - max(0, r - remainder) (read_HPC_row.cpp:255-266).
// Columns stay global (make_local_matrix localises them, as in the reference).
//
// The file is read once into memory and tokenised with strtol/strtod (the
// reference's fscanf per token is the same conversion, glibc correctly rounds
// both), so a 100^3 system parses in about a second.
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/HPC_Sparse_Matrix.hpp"
#include "../../include/hpccg_hip.h"

namespace hpccg {
int set_error_message(int code, const char* msg);
}

namespace {

int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int set_err(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return hpccg::set_error_message(code, buf);
}

struct Tokens {
    const char* p;
    const char* end;
    bool ok = true;

    void skip()
    {
        while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) p++;
    }
    long long next_int()
    {
        skip();
        char* e = nullptr;
        errno = 0;
        const long long v = std::strtoll(p, &e, 10);
        if (e == p || errno) ok = false;
        p = e ? e : p;
        return v;
    }
    double next_double()
    {
        skip();
        char* e = nullptr;
        const double v = std::strtod(p, &e);
        if (e == p) ok = false;
        p = e ? e : p;
        return v;
    }
};

}  // namespace

extern "C" int hpccg_read_HPC_row(const char* data_file, int rank, int size, HPC_Sparse_Matrix** Aout,
                                  double** xout, double** bout, double** xexout)
{
    if (!data_file || !Aout || !xout || !bout || !xexout || size < 1 || rank < 0 || rank >= size)
        return set_err(HPCCG_HIP_EINVAL, "read_HPC_row: bad argument");
    FILE* f = std::fopen(data_file, "rb");
    if (!f) return set_err(HPCCG_HIP_EINVAL, "Error: Cannot open file: %s", data_file);
    std::string buf;
    {
        std::fseek(f, 0, SEEK_END);
        const long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        buf.resize(sz > 0 ? (size_t)sz : 0);
        const size_t got = sz > 0 ? std::fread(&buf[0], 1, (size_t)sz, f) : 0;
        std::fclose(f);
        if ((long)got != sz) return set_err(HPCCG_HIP_EINVAL, "read_HPC_row: short read of %s", data_file);
        buf.push_back('\0');
    }
    Tokens t{buf.data(), buf.data() + buf.size() - 1};
    const long long total_nrow = t.next_int();
    const long long total_nnz = t.next_int();
    if (!t.ok || total_nrow < 1 || total_nrow >= (1LL << 31) || total_nnz < 0)
        return set_err(HPCCG_HIP_EINVAL, "read_HPC_row: bad header in %s", data_file);
    const int n = (int)total_nrow;
    const int chunksize = n / size, remainder = n % size;
    const int mp = chunksize + (rank < remainder ? 1 : 0);
    int off = rank * (chunksize + 1);
    if (rank > remainder) off -= rank - remainder;
    const int start_row = off, stop_row = off + mp - 1;

    std::vector<int> nnz_in_row(mp > 0 ? mp : 1);
    long long local_nnz = 0;
    for (int i = 0; i < n; i++) {
        const long long l = t.next_int();
        if (!t.ok || l < 0) return set_err(HPCCG_HIP_EINVAL, "read_HPC_row: bad row length, row %d", i);
        if (i >= start_row && i <= stop_row) {
            nnz_in_row[i - start_row] = (int)l;
            local_nnz += l;
        }
    }
    auto* A = new HPC_Sparse_Matrix();
    std::memset(A, 0, sizeof *A);
    A->nnz_in_row = new int[mp > 0 ? mp : 1];
    A->ptr_to_vals_in_row = new double*[mp > 0 ? mp : 1];
    A->ptr_to_inds_in_row = new int*[mp > 0 ? mp : 1];
    A->ptr_to_diags = new double*[mp > 0 ? mp : 1];
    A->list_of_vals = new double[local_nnz > 0 ? local_nnz : 1];
    A->list_of_inds = new int[local_nnz > 0 ? local_nnz : 1];
    auto* x = new double[mp > 0 ? mp : 1];
    auto* b = new double[mp > 0 ? mp : 1];
    auto* xe = new double[mp > 0 ? mp : 1];
    auto fail = [&](const char* what, int row) {
        hpccg_free_problem(A, x, b, xe);
        return set_err(HPCCG_HIP_EINVAL, "read_HPC_row: %s, row %d of %s", what, row, data_file);
    };
    long long pos = 0;
    for (int i = 0; i < mp; i++) {
        A->nnz_in_row[i] = nnz_in_row[i];
        A->ptr_to_vals_in_row[i] = A->list_of_vals + pos;
        A->ptr_to_inds_in_row[i] = A->list_of_inds + pos;
        A->ptr_to_diags[i] = nullptr;
        pos += nnz_in_row[i];
    }
    for (int i = 0; i < n; i++) {
        const long long cur = t.next_int();
        const bool mine = i >= start_row && i <= stop_row;
        if (!t.ok || (mine && cur != nnz_in_row[i - start_row])) return fail("entry count mismatch", i);
        for (long long j = 0; j < cur; j++) {
            const double v = t.next_double();
            const long long c = t.next_int();
            if (!t.ok || c < 0 || c >= total_nrow) return fail("bad entry", i);
            if (mine) {
                const int li = i - start_row;
                A->ptr_to_vals_in_row[li][j] = v;
                A->ptr_to_inds_in_row[li][j] = (int)c;
                if (c == i) A->ptr_to_diags[li] = &A->ptr_to_vals_in_row[li][j];
            }
        }
    }
    for (int i = 0; i < n; i++) {
        const double xt = t.next_double(), bt = t.next_double(), xxt = t.next_double();
        if (!t.ok) return fail("bad x b xexact line", i);
        if (i >= start_row && i <= stop_row) {
            x[i - start_row] = xt;
            b[i - start_row] = bt;
            xe[i - start_row] = xxt;
        }
    }
    A->title = nullptr;
    A->start_row = start_row;
    A->stop_row = stop_row;
    A->total_nrow = n;
    A->total_nnz = total_nnz;
    A->local_nrow = mp;
    A->local_ncol = mp;
    A->local_nnz = (int)local_nnz;
    *Aout = A;
    *xout = x;
    *bout = b;
    *xexout = xe;
    return 0;
}

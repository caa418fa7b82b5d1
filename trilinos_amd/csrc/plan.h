// Host-side index maps and import plans (bit-exact restatement of Epetra's rules).
#pragma once

#include <string>
#include <vector>

#include "internal.h"

namespace migmres {

void uniform_map(long long n_global, int nranks, int rank, long long *first, int *n_local);
int owner_of(long long gid, long long n_global, int nranks);
void epetra_shell_sort(std::vector<int> &keys, std::vector<long long> *c1, std::vector<int> *c2);

std::vector<long long> make_colmap(long long n_global, int nranks, long long first, int n_local,
                                   const long long *rowptr, const long long *gcols);

struct RemotePlan {
  int num_same = 0;
  std::vector<int> permute_to, permute_from;
  std::vector<int> remote_lids, remote_pids;
  std::vector<long long> remote_gids;
};

RemotePlan make_remotes(long long n_global, int nranks, long long first, int n_local,
                        const long long *colmap, int n_cols);

void local_crs(int n_local, const long long *rowptr, const long long *gcols, const double *vals,
               const long long *colmap, int n_cols, long long first, int *lcols_out,
               double *vals_out);

void galeri_rows(const std::string &kind, int nx, int ny, int nz, long long first, int n_local,
                 std::vector<long long> &rowptr, std::vector<long long> &gcols,
                 std::vector<double> &vals);

}  // namespace migmres

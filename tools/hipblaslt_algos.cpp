// Lists hipBLASLt bf16 GEMM solutions (index -> kernel name) so the TunableOp choices in
// gigapath/tuned/tunableop_results.csv ("Gemm_Hipblaslt_<index>") can be told apart: stream-K
// kernels carry "_SK" in their names.  Usage: tools/hipblaslt_algos [index ...]
// (no indices: every solution).  Build: hipcc --offload-arch=gfx950 -O2 tools/hipblaslt_algos.cpp
//   -lhipblaslt -o tools/hipblaslt_algos
// NOTE: this links /opt/rocm's hipBLASLt, whose solution indices are NOT the ones TunableOp records:
// PyTorch bundles its own hipBLASLt build (torch/lib, with rocRoller dependencies this tool cannot
// link), so the ids in gigapath/tuned/tunableop_results.csv resolve to NOT_FOUND here.
#include <hipblaslt/hipblaslt-ext.hpp>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  std::set<int> want;
  for (int i = 1; i < argc; ++i) want.insert(atoi(argv[i]));
  hipblasLtHandle_t h;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) { fprintf(stderr, "hipblasLtCreate failed\n"); return 1; }
  if (!want.empty()) {       // the given solution indices (TunableOp's "Gemm_Hipblaslt_<index>"), looked up directly
    {                        // getAllAlgos loads the bf16 solution libraries the index lookup searches
      std::vector<hipblasLtMatmulHeuristicResult_t> all;
      for (auto oa : {HIPBLAS_OP_N, HIPBLAS_OP_T})
        for (auto ob : {HIPBLAS_OP_N, HIPBLAS_OP_T})
          hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, oa, ob, HIP_R_16BF, HIP_R_16BF,
                                     HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all);
    }
    for (int idx : want) {
      std::vector<int> one{idx};
      std::vector<hipblasLtMatmulHeuristicResult_t> res;
      if (hipblaslt_ext::getAlgosFromIndex(h, one, res) != HIPBLAS_STATUS_SUCCESS || res.empty()) {
        printf("%d NOT_FOUND\n", idx);
        continue;
      }
      const std::string k = hipblaslt_ext::getKernelNameFromAlgo(h, res[0].algo);
      const bool sk = k.find("_SK") != std::string::npos && k.find("_SK0_") == std::string::npos;
      printf("%d %s %s\n", idx, sk ? "STREAMK" : "dataparallel", k.c_str());
    }
    hipblasLtDestroy(h);
    return 0;
  }
  const hipblasOperation_t ops[2] = {HIPBLAS_OP_N, HIPBLAS_OP_T};
  std::set<int> seen;
  for (auto oa : ops)
    for (auto ob : ops) {
      std::vector<hipblasLtMatmulHeuristicResult_t> res;
      if (hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, oa, ob, HIP_R_16BF, HIP_R_16BF,
                                     HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, res) != HIPBLAS_STATUS_SUCCESS)
        continue;
      for (auto& r : res) {
        const int idx = hipblaslt_ext::getIndexFromAlgo(r.algo);
        if (seen.count(idx) || (!want.empty() && !want.count(idx))) continue;
        seen.insert(idx);
        const std::string k = hipblaslt_ext::getKernelNameFromAlgo(h, r.algo);
        printf("%d %s %s%s\n", idx, k.find("_SK") != std::string::npos ? "STREAMK" : "dataparallel", k.c_str(),
               oa == HIPBLAS_OP_T && ob == HIPBLAS_OP_N ? " [TN]" : "");
      }
    }
  hipblasLtDestroy(h);
  return 0;
}

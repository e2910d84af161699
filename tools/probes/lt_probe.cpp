// Which hipBLASLt epilogues have bf16 kernels on this GPU?  Prints the number of
// heuristic candidates per (epilogue, bias type, aux type) for the GPT-2 MLP shape.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>

int main() {
  hipblasLtHandle_t h;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) { printf("create failed\n"); return 1; }
  const int64_t M = 20480, N = 3072, K = 768;
  struct E { const char* name; hipblasLtEpilogue_t e; } eps[] = {
      {"DEFAULT", HIPBLASLT_EPILOGUE_DEFAULT}, {"BIAS", HIPBLASLT_EPILOGUE_BIAS}, {"GELU", HIPBLASLT_EPILOGUE_GELU},
      {"GELU_BIAS", HIPBLASLT_EPILOGUE_GELU_BIAS}, {"GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX},
      {"GELU_AUX_BIAS", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS}, {"DGELU", HIPBLASLT_EPILOGUE_DGELU},
      {"DGELU_BGRAD", HIPBLASLT_EPILOGUE_DGELU_BGRAD}, {"BGRADA", HIPBLASLT_EPILOGUE_BGRADA},
      {"BGRADB", HIPBLASLT_EPILOGUE_BGRADB}};
  int types[] = {-1, HIP_R_16BF, HIP_R_32F};
  for (int ta = 0; ta < 2; ++ta)
  for (auto& e : eps)
    for (int bt : types)
      for (int at : types) {
        hipblasLtMatmulDesc_t d;
        hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F);
        int32_t opA = ta ? HIPBLAS_OP_N : HIPBLAS_OP_T, opB = HIPBLAS_OP_N;
        hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, 4);
        hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, 4);
        hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e.e, sizeof(e.e));
        if (bt >= 0) hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, 4);
        int64_t ld = N;
        hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, 8);
        if (at >= 0) hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, 4);
        hipblasLtMatrixLayout_t la, lb, lc;
        if (ta) hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, N, K, N);
        else hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K);
        hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K);
        hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, N, M, N);
        hipblasLtMatmulPreference_t pref;
        hipblasLtMatmulPreferenceCreate(&pref);
        uint64_t ws = 64ull << 20;
        hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, 8);
        hipblasLtMatmulHeuristicResult_t r[16];
        int got = 0;
        hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, lc, lc, pref, 16, r, &got);
        printf("%s %-14s bias=%3d aux=%3d status=%d cand=%d\n", ta ? "NN" : "TN", e.name, bt, at, (int)s, got);
        hipblasLtMatmulPreferenceDestroy(pref);
        hipblasLtMatrixLayoutDestroy(la); hipblasLtMatrixLayoutDestroy(lb); hipblasLtMatrixLayoutDestroy(lc);
        hipblasLtMatmulDescDestroy(d);
      }
  return 0;
}

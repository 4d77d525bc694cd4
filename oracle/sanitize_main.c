/* sanitize_main.c — drives every entry point of the CPU oracle (ldpc_oracle.c) on random graphs, including
 * degenerate ones (empty checks, unconnected variables, degree-1 checks, a lone edge), for the
 * -fsanitize=address,undefined build in tests/test_sanitizers.py.  TEST INFRASTRUCTURE ONLY. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define GRAPH_ARGS int m, int n, int E, const int32_t *row_ptr, const int32_t *col_idx, \
                   const int32_t *var_ptr, const int32_t *var_edges
int oracle_sp_f32(GRAPH_ARGS, const float* llr, int64_t B, int iters, float clamp, float* p1, float* z,
                  uint8_t* bits, float* trace, int early_stop, int32_t* iters_used, const void* w_vn,
                  const void* w_lw, const void* w_fin, const void* w_flw, int stable);
int oracle_sp_f64(GRAPH_ARGS, const double* llr, int64_t B, int iters, double clamp, double* p1, double* z,
                  uint8_t* bits, const void* w_vn, const void* w_lw, const void* w_fin, const void* w_flw);
int oracle_ms_f32(GRAPH_ARGS, const float* llr, int64_t B, int iters, float clamp, float alpha, float beta,
                  int early_stop, float* p1, float* z, uint8_t* bits, int32_t* iters_used);
int oracle_qms(GRAPH_ARGS, const int8_t* qllr, int64_t B, int iters, int qmax, int app_max, int beta,
               int early_stop, int16_t* app_out, uint8_t* bits, int32_t* iters_used);

static uint64_t st = 88172645463325252ull;
static uint32_t rnd(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (uint32_t)st; }
static double gauss(void) {
    const double u = (rnd() + 1.0) / 4294967297.0, v = (rnd() + 1.0) / 4294967297.0;
    return sqrt(-2.0 * log(u)) * cos(6.283185307179586 * v);
}

/* random m x n graph with density p; CSR (check order) and the var-order edge list, exactly sized */
static int run_graph(int m, int n, double p, int B) {
    uint8_t* H = calloc((size_t)m * n, 1);
    int E = 0;
    for (int i = 0; i < m * n; ++i) if ((rnd() % 10000) < p * 10000) { H[i] = 1; ++E; }
    int32_t* row_ptr = malloc(sizeof(int32_t) * (m + 1));
    int32_t* col_idx = malloc(sizeof(int32_t) * (E ? E : 1));
    int32_t* var_ptr = malloc(sizeof(int32_t) * (n + 1));
    int32_t* var_edges = malloc(sizeof(int32_t) * (E ? E : 1));
    int e = 0;
    for (int c = 0; c < m; ++c) {
        row_ptr[c] = e;
        for (int v = 0; v < n; ++v) if (H[c * n + v]) col_idx[e++] = v;
    }
    row_ptr[m] = e;
    int k = 0;
    for (int v = 0; v < n; ++v) {
        var_ptr[v] = k;
        for (int c = 0; c < m; ++c)
            for (int f = row_ptr[c]; f < row_ptr[c + 1]; ++f) if (col_idx[f] == v) var_edges[k++] = f;
    }
    var_ptr[n] = k;
    const size_t bn = (size_t)B * n;
    float* llr = malloc(sizeof(float) * bn);
    double* llr64 = malloc(sizeof(double) * bn);
    int8_t* q = malloc(bn);
    for (size_t i = 0; i < bn; ++i) {
        const double x = (rnd() % 16 == 0) ? 0.0 : 2.0 + 3.0 * gauss();  /* zeros: ties everywhere */
        llr[i] = (float)x;
        llr64[i] = x;
        q[i] = (int8_t)(x > 15 ? 15 : (x < -15 ? -15 : (int)lrint(x)));
    }
    float* p1 = malloc(sizeof(float) * bn);
    float* z = malloc(sizeof(float) * bn);
    double* p64 = malloc(sizeof(double) * bn);
    double* z64 = malloc(sizeof(double) * bn);
    uint8_t* bits = malloc(bn);
    int16_t* app = malloc(sizeof(int16_t) * bn);
    int32_t* used = malloc(sizeof(int32_t) * B);
    const int iters = 6;
    float* trace = malloc(sizeof(float) * (size_t)iters * B * (E ? E : 1));
    /* weights in the compact layout: W = sum d_v^2 per iteration */
    int64_t W = 0;
    for (int v = 0; v < n; ++v) { const int64_t d = var_ptr[v + 1] - var_ptr[v]; W += d * d; }
    float* wvn = malloc(sizeof(float) * (size_t)(iters * W + 1));
    float* wlw = malloc(sizeof(float) * (size_t)iters * n);
    float* wfin = malloc(sizeof(float) * (size_t)(E + 1));
    float* wflw = malloc(sizeof(float) * (size_t)n);
    for (int64_t i = 0; i < iters * W; ++i) wvn[i] = 0.5f + (rnd() % 1000) / 1000.0f;
    for (int i = 0; i < iters * n; ++i) wlw[i] = 0.5f + (rnd() % 1000) / 1000.0f;
    for (int i = 0; i < E; ++i) wfin[i] = 0.5f + (rnd() % 1000) / 1000.0f;
    for (int i = 0; i < n; ++i) wflw[i] = 0.5f + (rnd() % 1000) / 1000.0f;
    int rc = 0;
    for (int stable = 0; stable < 2; ++stable) {
        rc |= oracle_sp_f32(m, n, E, row_ptr, col_idx, var_ptr, var_edges, llr, B, iters, 10.0f, p1, z, bits, trace, 0,
                            used, NULL, NULL, NULL, NULL, stable);
        rc |= oracle_sp_f32(m, n, E, row_ptr, col_idx, var_ptr, var_edges, llr, B, 20, 20.0f, p1, z, bits, NULL, 1,
                            used, NULL, NULL, NULL, NULL, stable);
        rc |= oracle_sp_f32(m, n, E, row_ptr, col_idx, var_ptr, var_edges, llr, B, iters, 100.0f, p1, z, bits, NULL, 0,
                            NULL, wvn, wlw, wfin, wflw, stable);
    }
    rc |= oracle_sp_f64(m, n, E, row_ptr, col_idx, var_ptr, var_edges, llr64, B, iters, 10.0, p64, z64, bits, NULL,
                        NULL, NULL, NULL);
    rc |= oracle_ms_f32(m, n, E, row_ptr, col_idx, var_ptr, var_edges, llr, B, 20, 20.0f, 0.75f, 0.5f, 1, p1, z, bits,
                        used);
    rc |= oracle_qms(m, n, E, row_ptr, col_idx, var_ptr, var_edges, q, B, 20, 15, 127, 1, 1, app, bits, used);
    free(H); free(row_ptr); free(col_idx); free(var_ptr); free(var_edges); free(llr); free(llr64); free(q);
    free(p1); free(z); free(p64); free(z64); free(bits); free(app); free(used); free(trace);
    free(wvn); free(wlw); free(wfin); free(wflw);
    return rc;
}

int main(void) {
    int rc = 0;
    rc |= run_graph(12, 24, 0.25, 9);   /* dense-ish, several empty rows/columns likely */
    rc |= run_graph(30, 60, 0.06, 17);  /* sparse: degree-0/1/2 checks and variables */
    rc |= run_graph(1, 1, 1.0, 3);      /* one edge: a degree-1 check */
    rc |= run_graph(5, 7, 0.0, 4);      /* no edges at all */
    rc |= run_graph(40, 80, 0.5, 5);    /* long rows (d ~ 40) */
    printf("oracle sanitize: %s\n", rc ? "FAILED" : "ok");
    return rc ? 1 : 0;
}

/* A plain C99 consumer of include/pgh_api.h that closes a cycle on the GPU: what a cgo / JNI /
 * N-API binding of libpygrid_hip would do.  tests/test_gpu_group.py writes the inputs (MNIST
 * 784-392-10 synthetic diffs + checkpoint, oracle/gen_golden.py) and checks the outputs against
 * the golden SHA-256 of tests/golden/mnist_synth.json.
 *
 *   c_abi_gpu_close IN OUT N_GPUS [DEVICE ...]
 *   IN : int32 n_tensors, int32 n_clients, int64 numel[n_tensors], f32 diffs[n_clients][P], f32 ckpt[P]
 *   OUT: f32 mean[P] (cycle_manager.py:276-296), f32 iterative[P] (:266-269 + the notebook's plan)
 * N_GPUS 1 uses pgh_create(DEVICE); more use pgh_create_group (the devices may repeat). */
#include <stdio.h>
#include <stdlib.h>

#include "pgh_api.h"

#define CHECK(call)                                                                             \
    do {                                                                                        \
        int rc_ = (call);                                                                       \
        if (rc_ != PGH_OK) {                                                                    \
            fprintf(stderr, "%s -> %d: %s\n", #call, rc_, pgh_last_error(ctx));                 \
            return 2;                                                                           \
        }                                                                                       \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 4) return 1;
    const int n_gpus = atoi(argv[3]);
    int devices[64];
    for (int i = 0; i < n_gpus && i < 64; ++i) devices[i] = argc > 4 + i ? atoi(argv[4 + i]) : 0;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    int32_t hdr[2];
    if (fread(hdr, 4, 2, f) != 2) return 3;
    const int T = hdr[0], N = hdr[1];
    int64_t* numel = malloc(sizeof(int64_t) * (size_t)T);
    if (fread(numel, 8, (size_t)T, f) != (size_t)T) return 3;
    int64_t P = 0;
    for (int t = 0; t < T; ++t) P += numel[t];
    float* diffs = malloc(sizeof(float) * (size_t)(N * P));
    float* ckpt = malloc(sizeof(float) * (size_t)P);
    float* out = malloc(sizeof(float) * (size_t)P);
    if (fread(diffs, 4, (size_t)(N * P), f) != (size_t)(N * P) || fread(ckpt, 4, (size_t)P, f) != (size_t)P) return 3;
    fclose(f);

    pgh_ctx* ctx = NULL;
    if (n_gpus == 1) CHECK(pgh_create(devices[0], 0, &ctx));
    else CHECK(pgh_create_group(n_gpus, devices, 0, &ctx));
    int g = 0;
    CHECK(pgh_group_size(ctx, &g));
    if (g != n_gpus) return 4;
    CHECK(pgh_set_layout(ctx, T, numel));
    CHECK(pgh_reserve(ctx, N, PGH_F32, 1));
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 5;
    const int modes[2] = {PGH_MEAN, PGH_ITERATIVE_MEAN};
    for (int m = 0; m < 2; ++m) {
        CHECK(pgh_reset(ctx));
        for (int c = 0; c < N; ++c)
            CHECK(pgh_ingest_raw(ctx, c, diffs + (size_t)c * (size_t)P, sizeof(float) * (size_t)P, PGH_F32));
        CHECK(pgh_fedavg(ctx, modes[m], ckpt, out));
        if (fwrite(out, 4, (size_t)P, o) != (size_t)P) return 5;
    }
    fclose(o);
    pgh_stats_t st;
    CHECK(pgh_stats(ctx, &st));
    printf("ok gpus=%d P=%lld launches=%llu\n", g, (long long)st.p_shard, (unsigned long long)st.kernel_launches);
    pgh_destroy(ctx);
    free(numel);
    free(diffs);
    free(ckpt);
    free(out);
    return 0;
}

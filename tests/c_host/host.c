/* A C99 host of the C ABI (include/mbots.h), as a non-Python caller of the
 * reference's Manager surface would be (src/entry/mgr.hpp:10-68): create a
 * manager in MBOTS_EXEC_CPU mode, step / shift it with the identity-keyed
 * action stream, and print a digest of the exported views.
 * tests/test_c_host.py builds it with gcc -std=c99 -pedantic -Werror and
 * compares the digest with the same calls made through madrona_bots; built
 * with -DMBOTS_HOST_HIP (and the HIP runtime) it also runs MBOTS_EXEC_HIP
 * (argument "hip"), copying each device view to the host for the digest. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mbots.h"
#ifdef MBOTS_HOST_HIP
#include <hip/hip_runtime_api.h>
#endif

#define CHECK(call)                                                              \
    do {                                                                         \
        int rc_ = (call);                                                        \
        if (rc_ < 0) {                                                           \
            fprintf(stderr, "%s: %d %s\n", #call, rc_, mbots_last_error());      \
            return 1;                                                            \
        }                                                                        \
    } while (0)

static uint64_t fnv1a(const void *p, size_t n, uint64_t h)
{
    const unsigned char *b = (const unsigned char *)p;
    size_t i;
    for (i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

static size_t elem_size(int32_t dtype)
{
    return dtype == MBOTS_DTYPE_UINT8 || dtype == MBOTS_DTYPE_INT8 ? 1u : 4u;
}

int main(int argc, char **argv)
{
    const uint32_t worlds = argc > 1 ? (uint32_t)atoi(argv[1]) : 16u;
    const uint32_t steps = argc > 2 ? (uint32_t)atoi(argv[2]) : 6u;
    const int32_t mode = argc > 3 && strcmp(argv[3], "hip") == 0 ? MBOTS_EXEC_HIP : MBOTS_EXEC_CPU;
    static const int32_t ids[] = {MBOTS_EXPORT_ACTION, MBOTS_EXPORT_REWARD, MBOTS_EXPORT_POSITION,
                                  MBOTS_EXPORT_PREV_POSITION, MBOTS_EXPORT_HEALTH,
                                  MBOTS_EXPORT_SURROUNDING, MBOTS_EXPORT_SENSOR_SEMANTIC,
                                  MBOTS_EXPORT_PREV_SENSOR_SEMANTIC, MBOTS_EXPORT_STATS,
                                  MBOTS_EXPORT_SPECIES_COUNT};
    mbots_config cfg;
    mbots_handle *h = NULL;
    mbots_tensor t;
    uint32_t n = 0, s, k;
    uint64_t digest = 1469598103934665603ull;
    int rc;

    /* a bad config is refused before any work, with a message */
    memset(&cfg, 0, sizeof(cfg));
    cfg.sensor_size = 32;
    cfg.exec_mode = MBOTS_EXEC_CPU;
    rc = mbots_create(&cfg, &h);
    if (rc != MBOTS_E_INVALID || h != NULL || mbots_last_error()[0] == '\0') {
        fprintf(stderr, "num_worlds 0 accepted (%d)\n", rc);
        return 1;
    }

    cfg.num_worlds = worlds;
    cfg.exec_mode = mode;
    cfg.rand_seed = 69;
    cfg.init_num_agents_per_world = 32;
    CHECK(mbots_create(&cfg, &h));
    for (s = 0; s < steps; ++s) {
        CHECK(mbots_write_synthetic_actions(h, 1234u, s, 1, NULL));
        CHECK(mbots_step(h, NULL));
        if (s + 1 < steps) CHECK(mbots_shift_observations(h, NULL));
    }
    CHECK(mbots_num_agents(h, &n));
    for (k = 0; k < sizeof(ids) / sizeof(ids[0]); ++k) {
        size_t bytes;
        CHECK(mbots_export(h, ids[k], &t));
        bytes = (size_t)(t.dims[0] * t.dims[1]) * elem_size(t.dtype);
        if ((t.device == -1) != (mode == MBOTS_EXEC_CPU)) {
            fprintf(stderr, "export %d: device %d in mode %d\n", ids[k], t.device, mode);
            return 1;
        }
        if (t.device == -1) {
            digest = fnv1a(t.data, bytes, digest);
        } else {
#ifdef MBOTS_HOST_HIP
            /* mbots_export returns once the view's data is final */
            void *buf = malloc(bytes ? bytes : 1u);
            if (!buf || hipMemcpy(buf, t.data, bytes, hipMemcpyDeviceToHost) != hipSuccess) {
                fprintf(stderr, "hipMemcpy of export %d failed\n", ids[k]);
                return 1;
            }
            digest = fnv1a(buf, bytes, digest);
            free(buf);
#else
            fprintf(stderr, "built without MBOTS_HOST_HIP\n");
            return 1;
#endif
        }
    }
    CHECK(mbots_destroy(h));
    printf("agents %u digest %016llx\n", n, (unsigned long long)digest);
    return 0;
}

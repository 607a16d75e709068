/* Host AddressSanitizer check (scripts/asan_host.sh; CPU mode, no GPU): a
 * checkpoint saved at 128 slots restored into 1024 / 256 / 40-slot managers
 * and back, stepping in between, and mbots_max_population. */
#include <stdio.h>
#include <stdlib.h>
#include "mbots.h"
#define CHECK(c) do { int r_ = (c); if (r_ < 0) { fprintf(stderr, "%s: %d %s\n", #c, r_, mbots_last_error()); return 1; } } while (0)
static int run(mbots_handle *h, int from, int to) {
    for (int t = from; t < to; ++t) {
        CHECK(mbots_write_synthetic_actions(h, 1234, t, 1, NULL));
        int rc = mbots_step(h, NULL); if (rc < 0) { fprintf(stderr, "step %d\n", rc); return 1; }
        CHECK(mbots_shift_observations(h, NULL));
    }
    return 0;
}
int main(void) {
    mbots_config c = {0};
    c.gpu_id = 0; c.num_worlds = 12; c.rand_seed = 69; c.init_num_agents_per_world = 32;
    c.sensor_size = 32; c.agent_capacity = 128; c.exec_mode = MBOTS_EXEC_CPU;
    mbots_handle *a = NULL; CHECK(mbots_create(&c, &a));
    if (run(a, 0, 8)) return 1;
    uint64_t n = 0; CHECK(mbots_checkpoint_size(a, &n));
    void *blob = malloc(n); CHECK(mbots_save_checkpoint(a, blob, n));
    unsigned caps[3] = {1024, 256, 40};
    for (int i = 0; i < 3; ++i) {
        mbots_config d = c; d.agent_capacity = caps[i];
        mbots_handle *b = NULL; CHECK(mbots_create(&d, &b));
        int rc = mbots_load_checkpoint(b, blob, n);
        printf("cap %u load rc %d %s\n", caps[i], rc, rc ? mbots_last_error() : "");
        if (rc == 0 && run(b, 8, 14)) return 1;
        uint32_t mp = 0; CHECK(mbots_max_population(b, &mp)); printf("  max population %u\n", mp);
        /* and back: save from the other class, load into 128 */
        uint64_t m = 0; CHECK(mbots_checkpoint_size(b, &m));
        void *b2 = malloc(m); CHECK(mbots_save_checkpoint(b, b2, m));
        mbots_handle *e = NULL; CHECK(mbots_create(&c, &e));
        rc = mbots_load_checkpoint(e, b2, m); printf("  back to 128: rc %d\n", rc);
        free(b2); mbots_destroy(e); mbots_destroy(b);
    }
    free(blob); mbots_destroy(a);
    puts("ok");
    return 0;
}

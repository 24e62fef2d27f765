/* CPU unit test of xsk_gpu_multi_process's all-or-nothing counter fold (xsk_gpu__multi_fold,
 * xsknet_amd/csrc/xsk_gpu_internal.h).  Built and run by tests/test_abi.py. */
#include <assert.h>
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include "../../xsknet_amd/csrc/xsk_gpu_internal.h"

int main(void) {
    struct xsk_gpu_stats st[3];
    memset(st, 0, sizeof st);
    for (int g = 0; g < 3; g++) {
        st[g].rx_packets = 10u + g;
        st[g].rx_bytes = 1000u * (g + 1);
        st[g].tx_packets = 5u + g;
        st[g].tx_bytes = 500u * (g + 1);
    }
    struct xsk_gpu_stats out = {7, 1, 2, 3, 4};
    int rc[3] = {0, 0, 0};
    assert(xsk_gpu__multi_fold(rc, st, 3, &out) == 0);
    assert(out.timestamp == 7 && out.rx_packets == 1 + 33 && out.rx_bytes == 2 + 6000 && out.tx_packets == 3 + 18 &&
           out.tx_bytes == 4 + 3000);
    /* one context fails (an injected error): nothing is added, the first error comes back */
    const struct xsk_gpu_stats before = out;
    rc[1] = -EIO;
    rc[2] = -EBUSY;
    assert(xsk_gpu__multi_fold(rc, st, 3, &out) == -EIO);
    assert(memcmp(&out, &before, sizeof out) == 0);
    rc[1] = 0;
    assert(xsk_gpu__multi_fold(rc, st, 3, &out) == -EBUSY);
    assert(memcmp(&out, &before, sizeof out) == 0);
    /* no stats pointer: the status alone */
    rc[2] = 0;
    assert(xsk_gpu__multi_fold(rc, st, 3, NULL) == 0);
    printf("multi fold ok\n");
    return 0;
}

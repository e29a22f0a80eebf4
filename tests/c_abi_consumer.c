/* A plain C99 consumer of include/pgh_api.h: compiled and linked against libpygrid_hip.so by
 * tests/test_abi.py (no GPU needed: it only exercises the host-only entry points and the error
 * path of context creation). */
#include <stdio.h>
#include <string.h>

#include "pgh_api.h"

int main(void) {
    if (pgh_abi_version() != PGH_ABI_VERSION) return 10;
    pgh_ctx* ctx = NULL;
    int n = -1;
    int rc = pgh_device_count(&n);
    if (n == 0 && pgh_create(0, 0, &ctx) == PGH_OK) return 11;   /* no GPU: creation must fail */
    if (n == 0 && strlen(pgh_last_error(NULL)) == 0) return 12;
    const char* b64 = "QUJDRA==";
    unsigned char out[8];
    size_t w = 0;
    if (pgh_b64_decode(b64, strlen(b64), out, &w, 1) != PGH_OK || w != 4 || memcmp(out, "ABCD", 4)) return 13;
    int nt = -1;
    if (pgh_state_scan((const uint8_t*)"", 0, 0, NULL, NULL, &nt) != PGH_OK || nt != 0) return 14;
    printf("ok %d %d\n", rc, n);
    return 0;
}

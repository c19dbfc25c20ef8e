/* tests/native/abi_c_consumer.c -- a plain C99 caller of the C ABI (include/oxen_hash.h), built with gcc
 * -std=c99 against liboxen_hash.so: the boundary a cgo / bindgen / Rust `extern "C"` block binds, used
 * with no C++ or HIP type on this side. Without a GPU it checks the library-level calls and that
 * context creation fails with OXH_ERR_NODEVICE (no CPU fallback); with one (argv[1] == "gpu") it hashes
 * the reference's known answer (repositories/data_frames/schemas.rs:131) and the SURVEY §8c vectors
 * through oxh_hash_buffers and oxh_hash_streams, formats them as MerkleHash Display does
 * (merkle_hash.rs:73-77) and checks every digest. Exit status 0 = all checks passed. */
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#include "../../include/oxen_hash.h"

static int failures = 0;
#define CHECK(cond)                                                       \
    do {                                                                  \
        if (!(cond)) {                                                    \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                   \
        }                                                                 \
    } while (0)

static const char* const kInputs[] = {"filestrlabelstrmin_xf64min_yf64widthi64heighti64", "", "hello",
                                      "File content 0"};
static const char* const kHex[] = {"b821946753334c083124fd563377d795", "99aa06d3014798d86001c324468d497f",
                                   "b5e9c1ad071b3e7fc779cfaa5e523818", "393ba5849f5590fc5985c4bbcec0003f"};
#define NKAT 4

int main(int argc, char** argv) {
    const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    char hex[33], dec[40];
    CHECK(oxh_abi_version() == OXH_ABI_VERSION);
    /* formatting: unpadded lowercase hex, u128 decimal */
    CHECK(oxh_format_hex(0x3124fd563377d795ull, 0xb821946753334c08ull, hex) == 32);
    CHECK(strcmp(hex, kHex[0]) == 0);
    CHECK(oxh_format_hex(0x1ull, 0x0ull, hex) == 1 && strcmp(hex, "1") == 0);
    CHECK(oxh_format_dec(12345ull, 0ull, dec) == 5 && strcmp(dec, "12345") == 0);
    CHECK(oxh_format_dec(0ull, 1ull, dec) == 20 && strcmp(dec, "18446744073709551616") == 0);
    /* argument errors before any device work */
    CHECK(oxh_ctx_create(0, 0, NULL) == OXH_ERR_INVALID);
    CHECK(oxh_ctx_create(0, (uint64_t)OXH_MAX_STAGING_BYTES + 1, NULL) == OXH_ERR_INVALID);
    CHECK(oxh_comm_unique_id(NULL) == OXH_ERR_INVALID);
    CHECK(oxh_ctx_destroy(NULL) == OXH_OK);
    oxh_ctx* ctx = NULL;
    const int rc = oxh_ctx_create(0, 1 << 20, &ctx);
    if (!gpu) {
        CHECK(rc == OXH_ERR_NODEVICE && ctx == NULL);  /* no CPU fallback */
        CHECK(strlen(oxh_last_error()) > 0);
        CHECK(oxh_comm_check(0) == OXH_ERR_NODEVICE);
    } else {
        CHECK(rc == OXH_OK && ctx != NULL);
        if (rc == OXH_OK) {
            const uint8_t* bufs[NKAT];
            uint64_t lens[NKAT], offs[NKAT], out[2 * NKAT], out2[2 * NKAT];
            char arena[256];
            uint64_t pos = 0;
            for (int i = 0; i < NKAT; ++i) {
                bufs[i] = (const uint8_t*)kInputs[i];
                lens[i] = strlen(kInputs[i]);
                offs[i] = pos;
                memcpy(arena + pos, kInputs[i], lens[i]);
                pos += lens[i];
            }
            CHECK(oxh_hash_buffers(ctx, bufs, lens, NKAT, out) == OXH_OK);
            CHECK(oxh_hash_streams(ctx, (const uint8_t*)arena, offs, lens, NKAT, out2) == OXH_OK);
            for (int i = 0; i < NKAT; ++i) {
                oxh_format_hex(out[2 * i], out[2 * i + 1], hex);
                CHECK(strcmp(hex, kHex[i]) == 0);
                CHECK(out2[2 * i] == out[2 * i] && out2[2 * i + 1] == out[2 * i + 1]);
            }
            CHECK(oxh_ctx_destroy(ctx) == OXH_OK);
        }
    }
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("abi_c_consumer: all checks passed (%s)\n", gpu ? "gpu" : "no device");
    return 0;
}

/*
 * rules_bin.c — binary prefix dumps for large rule and route sets.
 *
 * rules.json (firewall.c:276-323) costs a JSON object per rule and, in the
 * reference's reader, one fgets per line; at the 1M-entry sizes of BASELINE
 * configs[4] a flat binary file is the practical format.
 *
 * Layout (little-endian):
 *   offset 0   char     magic[4] = "CPRB"
 *          4   uint32_t version  = 1
 *          8   uint64_t n        number of records
 *         16   n records of 12 bytes, the cop_prefix layout:
 *              uint32_t ip (host order), uint32_t next_hop, uint8_t depth,
 *              uint8_t pad[3] (written 0, ignored on read)
 * Records are kept in file order: lpm_setup semantics (add in order, last
 * write wins, stop or skip at errors) apply to a binary file exactly as to
 * a JSON one.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cop_internal.h"

#define BIN_MAGIC "CPRB"
#define BIN_VERSION 1u
#define BIN_HDR 16u
#define BIN_REC 12u

_Static_assert(sizeof(cop_prefix) == BIN_REC, "cop_prefix must be the 12-byte record");

int cop_rules_write_bin(const char *path, const cop_prefix *rules, uint32_t n)
{
    if (!path || (n && !rules)) return -EINVAL;
    FILE *fp = fopen(path, "wb");
    if (!fp) return -errno;
    uint8_t hdr[BIN_HDR];
    uint32_t ver = BIN_VERSION;
    uint64_t cnt = n;
    memcpy(hdr, BIN_MAGIC, 4);
    memcpy(hdr + 4, &ver, 4);
    memcpy(hdr + 8, &cnt, 8);
    int ok = fwrite(hdr, 1, BIN_HDR, fp) == BIN_HDR;
    /* records with their pad bytes zeroed, in chunks */
    cop_prefix buf[4096];
    for (uint32_t i = 0; ok && i < n; i += 4096) {
        uint32_t k = n - i < 4096 ? n - i : 4096;
        for (uint32_t j = 0; j < k; j++) {
            memset(&buf[j], 0, sizeof(buf[j]));
            buf[j].ip = rules[i + j].ip;
            buf[j].next_hop = rules[i + j].next_hop;
            buf[j].depth = rules[i + j].depth;
        }
        ok = fwrite(buf, BIN_REC, k, fp) == k;
    }
    if (fclose(fp) != 0) ok = 0;
    return ok ? 0 : -EIO;
}

int cop_rules_load_bin(const char *path, cop_prefix **out, uint32_t *n)
{
    if (!path || !out || !n) return -EINVAL;
    *out = NULL;
    *n = 0;
    FILE *fp = fopen(path, "rb");
    if (!fp) return -ENOENT;
    uint8_t hdr[BIN_HDR];
    uint32_t ver;
    uint64_t cnt;
    int rc = 0;
    if (fread(hdr, 1, BIN_HDR, fp) != BIN_HDR || memcmp(hdr, BIN_MAGIC, 4) != 0) {
        rc = -EINVAL;
    } else {
        memcpy(&ver, hdr + 4, 4);
        memcpy(&cnt, hdr + 8, 8);
        if (ver != BIN_VERSION || cnt > 0xFFFFFFFFull) rc = -EINVAL;
    }
    /* the file must hold exactly cnt records */
    long want = 0;
    if (!rc) {
        want = (long)(BIN_HDR + cnt * BIN_REC);
        if (fseek(fp, 0, SEEK_END) != 0 || ftell(fp) != want || fseek(fp, BIN_HDR, SEEK_SET) != 0)
            rc = -EINVAL;
    }
    cop_prefix *r = NULL;
    if (!rc) {
        r = (cop_prefix *)malloc((size_t)(cnt ? cnt : 1) * BIN_REC);
        if (!r) rc = -ENOMEM;
        else if (cnt && fread(r, BIN_REC, (size_t)cnt, fp) != cnt) rc = -EIO;
    }
    fclose(fp);
    if (rc) {
        free(r);
        return rc;
    }
    for (uint64_t i = 0; i < cnt; i++) memset(r[i]._pad, 0, sizeof(r[i]._pad));
    *out = r;
    *n = (uint32_t)cnt;
    return 0;
}

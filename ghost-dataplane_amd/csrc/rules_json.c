/*
 * rules_json.c — rules.json loader/writer (host setup path).
 *
 * Restates setup_rules / fw_config_parse_file / fw_pkt_parse_ip
 * (firewall.c:32-55, 57-105, 276-323) without the vendored cJSON, with
 * cJSON 1.7.12's grammar (BOM, whitespace = any byte <= 32, strtod numbers
 * over [0-9+-.eE], raw control bytes in strings, invalid \u hex = 0,
 * trailing bytes after the root ignored); tests/test_ref_cjson.py pins it
 * to the reference's own cJSON build:
 *   - the root's children, in file order, are the rules
 *     (fw_config_get_item_count firewall.c:107-127 counts them);
 *   - keys are matched case-insensitively, first match wins
 *     (cJSON_GetObjectItem, cJSON.c:1811);
 *   - "ip" must be a string and goes through sscanf("%u.%u.%u.%u") with
 *     each byte masked & 0xff (RTE_IPV4, firewall.h:112);
 *   - "depth"/"action" take cJSON's valueint (number clamped to int,
 *     true -> 1, anything else 0) and are truncated to uint8 by the
 *     struct fw_rule fields (firewall.h:49-53).
 * Deviations (the reference's behaviour is undefined there): a missing key
 * or an unparsable ip is an error (-EINVAL) instead of rte_exit / an
 * uninitialised src_ip; lines of any length are accepted (the reference's
 * fgets into a 255-byte stack buffer overflows, firewall.c:72,95).
 */
#include <ctype.h>
#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cop_gpu.h"

enum jtype { J_NULL, J_FALSE, J_TRUE, J_NUMBER, J_STRING, J_ARRAY, J_OBJECT };

typedef struct jnode {
    enum jtype type;
    char *key;         /* member name when inside an object */
    char *str;         /* J_STRING */
    double num;        /* J_NUMBER */
    struct jnode *child, *next;
} jnode;

typedef struct {
    const char *p, *end;
    int depth;
} jparser;

static void jfree(jnode *n)
{
    while (n) {
        jnode *nx = n->next;
        jfree(n->child);
        free(n->key);
        free(n->str);
        free(n);
        n = nx;
    }
}

static void skip_ws(jparser *ps)
{
    /* cJSON's buffer_skip_whitespace: every byte <= 32 */
    while (ps->p < ps->end && (unsigned char)*ps->p <= 32) ps->p++;
}

static jnode *parse_value(jparser *ps);

/* cJSON parse_hex4: an invalid digit makes the whole value 0 */
static unsigned hex4(const char *s)
{
    unsigned v = 0;
    for (int i = 0; i < 4; i++) {
        char c = s[i];
        v <<= 4;
        if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
        else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
        else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
        else return 0;
    }
    return v;
}

/* cJSON parse_string: find the closing quote first (a backslash skips the
 * next byte), then decode the escapes inside [start, end); \u sequences
 * must fit before the closing quote. Control bytes are kept as they are. */
static char *parse_string(jparser *ps)
{
    if (ps->p >= ps->end || *ps->p != '"') return NULL;
    const char *q = ps->p + 1;
    while (q < ps->end && *q != '"') {
        if (*q == '\\') {
            if (q + 1 >= ps->end) return NULL;
            q++;
        }
        q++;
    }
    if (q >= ps->end) return NULL;
    const char *in = ps->p + 1, *end = q;
    char *out = (char *)malloc((size_t)(end - in) + 1);
    size_t len = 0;
    if (!out) return NULL;
    while (in < end) {
        if (*in != '\\') {
            out[len++] = *in++;
            continue;
        }
        unsigned cp;
        switch (in[1]) {
        case 'b': out[len++] = '\b'; in += 2; break;
        case 'f': out[len++] = '\f'; in += 2; break;
        case 'n': out[len++] = '\n'; in += 2; break;
        case 'r': out[len++] = '\r'; in += 2; break;
        case 't': out[len++] = '\t'; in += 2; break;
        case '"': case '\\': case '/': out[len++] = in[1]; in += 2; break;
        case 'u':
            if (end - in < 6) goto fail;
            cp = hex4(in + 2);
            if (cp >= 0xDC00 && cp <= 0xDFFF) goto fail;
            if (cp >= 0xD800 && cp <= 0xDBFF) {
                const char *sec = in + 6;
                if (end - sec < 6 || sec[0] != '\\' || sec[1] != 'u') goto fail;
                unsigned lo = hex4(sec + 2);
                if (lo < 0xDC00 || lo > 0xDFFF) goto fail;
                cp = 0x10000 + (((cp & 0x3FF) << 10) | (lo & 0x3FF));
                in += 12;
            } else {
                in += 6;
            }
            /* UTF-8; \u escapes expand to at most as many bytes as they take */
            if (cp < 0x80) {
                out[len++] = (char)cp;
            } else if (cp < 0x800) {
                out[len++] = (char)(0xC0 | (cp >> 6));
                out[len++] = (char)(0x80 | (cp & 0x3F));
            } else if (cp < 0x10000) {
                out[len++] = (char)(0xE0 | (cp >> 12));
                out[len++] = (char)(0x80 | ((cp >> 6) & 0x3F));
                out[len++] = (char)(0x80 | (cp & 0x3F));
            } else {
                out[len++] = (char)(0xF0 | (cp >> 18));
                out[len++] = (char)(0x80 | ((cp >> 12) & 0x3F));
                out[len++] = (char)(0x80 | ((cp >> 6) & 0x3F));
                out[len++] = (char)(0x80 | (cp & 0x3F));
            }
            break;
        default:
            goto fail;
        }
    }
    out[len] = 0;   /* a decoded \u0000 ends the C string, as in cJSON */
    ps->p = end + 1;
    return out;
fail:
    free(out);
    return NULL;
}

static jnode *new_node(enum jtype t)
{
    jnode *n = (jnode *)calloc(1, sizeof(jnode));
    if (n) n->type = t;
    return n;
}

static jnode *parse_container(jparser *ps, int is_obj)
{
    char close = is_obj ? '}' : ']';
    jnode *n = new_node(is_obj ? J_OBJECT : J_ARRAY), *tail = NULL;
    if (!n) return NULL;
    if (++ps->depth > 1000) goto fail; /* CJSON_NESTING_LIMIT */
    ps->p++;
    skip_ws(ps);
    if (ps->p < ps->end && *ps->p == close) {
        ps->p++;
        ps->depth--;
        return n;
    }
    for (;;) {
        char *key = NULL;
        skip_ws(ps);
        if (is_obj) {
            key = parse_string(ps);
            if (!key) goto fail;
            skip_ws(ps);
            if (ps->p >= ps->end || *ps->p != ':') {
                free(key);
                goto fail;
            }
            ps->p++;
            skip_ws(ps);
        }
        jnode *c = parse_value(ps);
        if (!c) {
            free(key);
            goto fail;
        }
        c->key = key;
        if (tail) tail->next = c;
        else n->child = c;
        tail = c;
        skip_ws(ps);
        if (ps->p >= ps->end) goto fail;
        if (*ps->p == ',') {
            ps->p++;
            continue;
        }
        if (*ps->p == close) {
            ps->p++;
            break;
        }
        goto fail;
    }
    ps->depth--;
    return n;
fail:
    jfree(n);
    return NULL;
}

static jnode *parse_value(jparser *ps)
{
    skip_ws(ps);
    if (ps->p >= ps->end) return NULL;
    size_t left = (size_t)(ps->end - ps->p);
    char c = *ps->p;
    if (left >= 4 && !strncmp(ps->p, "null", 4)) {
        ps->p += 4;
        return new_node(J_NULL);
    }
    if (left >= 5 && !strncmp(ps->p, "false", 5)) {
        ps->p += 5;
        return new_node(J_FALSE);
    }
    if (left >= 4 && !strncmp(ps->p, "true", 4)) {
        ps->p += 4;
        return new_node(J_TRUE);
    }
    if (c == '"') {
        char *s = parse_string(ps);
        if (!s) return NULL;
        jnode *n = new_node(J_STRING);
        if (!n) {
            free(s);
            return NULL;
        }
        n->str = s;
        return n;
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
        /* cJSON parse_number: take the run of [0-9+-eE.] and strtod it */
        char buf[64];
        size_t k = 0;
        while (ps->p + k < ps->end && k < sizeof(buf) - 1 &&
               strchr("0123456789+-eE.", ps->p[k]) && ps->p[k])
            k++;
        memcpy(buf, ps->p, k);
        buf[k] = 0;
        char *e;
        double d = strtod(buf, &e);
        if (e == buf) return NULL;
        ps->p += (e - buf);
        jnode *n = new_node(J_NUMBER);
        if (n) n->num = d;
        return n;
    }
    if (c == '[') return parse_container(ps, 0);
    if (c == '{') return parse_container(ps, 1);
    return NULL;
}

static int key_eq_ci(const char *a, const char *b)
{
    if (!a || !b) return 0;
    for (; *a && *b; a++, b++)
        if (tolower((unsigned char)*a) != tolower((unsigned char)*b)) return 0;
    return *a == *b;
}

static const jnode *get_item(const jnode *obj, const char *key)
{
    if (!obj || obj->type != J_OBJECT) return NULL;
    for (const jnode *c = obj->child; c; c = c->next)
        if (key_eq_ci(c->key, key)) return c;
    return NULL;
}

static int valueint(const jnode *n)
{
    if (n->type == J_TRUE) return 1;
    if (n->type != J_NUMBER) return 0;
    if (n->num >= INT_MAX) return INT_MAX;
    if (n->num <= (double)INT_MIN) return INT_MIN;
    return (int)n->num;
}

int cop_rules_load_json(const char *path, cop_prefix **out, uint32_t *n_out)
{
    if (!path || !*path || !out || !n_out) return -EINVAL;
    *out = NULL;
    *n_out = 0;
    FILE *fp = fopen(path, "rb");
    if (!fp) return -ENOENT;
    fseek(fp, 0L, SEEK_END);
    long len = ftell(fp);
    rewind(fp);
    if (len < 0) {
        fclose(fp);
        return -EIO;
    }
    char *buf = (char *)malloc((size_t)len + 1);
    if (!buf) {
        fclose(fp);
        return -ENOMEM;
    }
    size_t got = fread(buf, 1, (size_t)len, fp);
    fclose(fp);
    buf[got] = 0;
    /* the reference builds its buffer with fgets/strlen, so a NUL byte ends it */
    jparser ps = {buf, buf + strlen(buf), 0};
    /* cJSON skip_utf8_bom (cJSON_ParseWithOpts) */
    if (ps.end - ps.p >= 4 && !memcmp(ps.p, "\xEF\xBB\xBF", 3)) ps.p += 3;
    jnode *root = parse_value(&ps);
    free(buf);
    if (!root) return -EINVAL;

    uint32_t cnt = 0;
    for (jnode *c = root->child; c; c = c->next) cnt++;
    cop_prefix *rules = (cop_prefix *)calloc(cnt ? cnt : 1, sizeof(cop_prefix));
    if (!rules) {
        jfree(root);
        return -ENOMEM;
    }
    uint32_t i = 0;
    int rc = 0;
    for (jnode *c = root->child; c; c = c->next, i++) {
        const jnode *ip = get_item(c, "ip");
        const jnode *depth = get_item(c, "depth");
        const jnode *action = get_item(c, "action");
        if (!ip || !depth || !action || ip->type != J_STRING) {
            rc = -EINVAL;
            break;
        }
        unsigned int b[4];
        if (sscanf(ip->str, "%u.%u.%u.%u", &b[0], &b[1], &b[2], &b[3]) != 4) {
            rc = -EINVAL;
            break;
        }
        rules[i].ip = ((b[0] & 0xffu) << 24) | ((b[1] & 0xffu) << 16) | ((b[2] & 0xffu) << 8) |
                      (b[3] & 0xffu);
        rules[i].depth = (uint8_t)valueint(depth);
        rules[i].next_hop = (uint8_t)valueint(action);
    }
    jfree(root);
    if (rc) {
        free(rules);
        return rc;
    }
    *out = rules;
    *n_out = cnt;
    return 0;
}

void cop_rules_free(cop_prefix *rules)
{
    free(rules);
}

int cop_rules_write_json(const char *path, const cop_prefix *rules, uint32_t n)
{
    if (!path || (n && !rules)) return -EINVAL;
    FILE *fp = fopen(path, "w");
    if (!fp) return -errno;
    fprintf(fp, "{\n");
    for (uint32_t i = 0; i < n; i++) {
        uint32_t ip = rules[i].ip;
        fprintf(fp,
                "\t\"rule%u\": {\n\t\t\"ip\": \"%u.%u.%u.%u\",\n\t\t\"depth\": %u,\n"
                "\t\t\"action\": %u\n\t}%s\n",
                i + 1, (ip >> 24) & 0xFF, (ip >> 16) & 0xFF, (ip >> 8) & 0xFF, ip & 0xFF,
                (unsigned)rules[i].depth, (unsigned)rules[i].next_hop, i + 1 < n ? "," : "");
    }
    fprintf(fp, "}\n");
    return fclose(fp) ? -EIO : 0;
}

void cop_route_table_default(uint16_t *rt, uint32_t n_ports)
{
    /* read_config, init.c:40-84: the table is zero-initialised global
     * storage; entries 0..KNI_KTHREAD-1 get UINT16_MAX; vport i has IP
     * 192.167.10.(i+1) and routing_table[ip & 0xFFFF] = i. */
    memset(rt, 0, COP_ROUTING_TBL_SZ * sizeof(uint16_t));
    for (uint32_t i = 0; i < n_ports; i++) rt[i] = 0xFFFF;
    for (uint32_t i = 0; i < n_ports; i++) {
        uint32_t ip = (192u << 24) | (167u << 16) | (10u << 8) | ((i + 1) & 0xFFu);
        rt[ip & 0xFFFF] = (uint16_t)i;
    }
}

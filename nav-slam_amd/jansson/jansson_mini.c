/*
 * jansson_mini.c — the jansson subset declared in jansson.h (see there for
 * the exact semantics): a recursive-descent JSON parser over the whole input
 * held in memory, values reference counted like jansson's.
 *
 * Only the K1 plumbing links it (the reference src/main.c reads its L5 and
 * IMU frames through it, src/main.c:13-74,131-185); nothing on the GPU path
 * does.
 */
#include "jansson.h"

#include <errno.h>
#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

typedef struct { json_t j; json_int_t v; } jint;
typedef struct { json_t j; double v; } jreal;
typedef struct { json_t j; char *s; } jstr;
typedef struct { json_t j; size_t n, cap; json_t **v; } jarr;
typedef struct { json_t j; size_t n, cap; char **k; json_t **v; } jobj;

static json_t s_true = {JSON_TRUE, (size_t)-1};
static json_t s_false = {JSON_FALSE, (size_t)-1};
static json_t s_null = {JSON_NULL, (size_t)-1};

enum { kMaxDepth = 2048 }; /* jansson's JSON_PARSER_MAX_DEPTH */

typedef struct {
    const char *s, *p, *end, *line_start;
    int line;
    json_error_t *err;
    int failed;
} parser;

static void fail(parser *ps, const char *fmt, ...)
{
    if (ps->failed)
        return;
    ps->failed = 1;
    if (!ps->err)
        return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(ps->err->text, JSON_ERROR_TEXT_LENGTH, fmt, ap);
    va_end(ap);
    ps->err->line = ps->line;
    ps->err->column = (int)(ps->p - ps->line_start) + 1;
    ps->err->position = (int)(ps->p - ps->s);
}

static void skip_ws(parser *ps)
{
    while (ps->p < ps->end) {
        const char c = *ps->p;
        if (c == '\n') {
            ps->line++;
            ps->line_start = ps->p + 1;
        } else if (c != ' ' && c != '\t' && c != '\r') {
            break;
        }
        ps->p++;
    }
}

static json_t *alloc_value(size_t size, json_type t)
{
    json_t *j = calloc(1, size);
    if (j) {
        j->type = t;
        j->refcount = 1;
    }
    return j;
}

static int push(void ***v, size_t *n, size_t *cap, void *x)
{
    if (*n == *cap) {
        const size_t nc = *cap ? 2 * *cap : 8;
        void **nv = realloc(*v, nc * sizeof(void *));
        if (!nv)
            return -1;
        *v = nv;
        *cap = nc;
    }
    (*v)[(*n)++] = x;
    return 0;
}

static int hexval(char c)
{
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static int hex4(parser *ps, const char *p, unsigned *out)
{
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
        const int h = p + i < ps->end ? hexval(p[i]) : -1;
        if (h < 0)
            return -1;
        v = v * 16 + (unsigned)h;
    }
    *out = v;
    return 0;
}

static char *put_utf8(char *o, unsigned cp)
{
    if (cp < 0x80) {
        *o++ = (char)cp;
    } else if (cp < 0x800) {
        *o++ = (char)(0xC0 | (cp >> 6));
        *o++ = (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
        *o++ = (char)(0xE0 | (cp >> 12));
        *o++ = (char)(0x80 | ((cp >> 6) & 0x3F));
        *o++ = (char)(0x80 | (cp & 0x3F));
    } else {
        *o++ = (char)(0xF0 | (cp >> 18));
        *o++ = (char)(0x80 | ((cp >> 12) & 0x3F));
        *o++ = (char)(0x80 | ((cp >> 6) & 0x3F));
        *o++ = (char)(0x80 | (cp & 0x3F));
    }
    return o;
}

/* ps->p at the opening quote. Returns a malloc'd, NUL-terminated string and
 * its byte length (which may include \u0000 bytes) in *len. */
static char *parse_string_raw(parser *ps, size_t *len)
{
    const char *q = ps->p + 1;
    while (q < ps->end && *q != '"') /* closing quote: output <= input */
        q += (*q == '\\' && q + 1 < ps->end) ? 2 : 1;
    if (q >= ps->end) {
        fail(ps, "premature end of input");
        return NULL;
    }
    char *out = malloc((size_t)(q - ps->p) + 1), *o = out;
    if (!out) {
        fail(ps, "out of memory");
        return NULL;
    }
    const char *p = ps->p + 1;
    while (p < q) {
        const unsigned char c = (unsigned char)*p;
        if (c < 0x20) {
            ps->p = p;
            fail(ps, "control character 0x%x", c);
            free(out);
            return NULL;
        }
        if (c != '\\') {
            *o++ = (char)c;
            p++;
            continue;
        }
        const char e = p[1];
        p += 2;
        switch (e) {
        case '"': *o++ = '"'; break;
        case '\\': *o++ = '\\'; break;
        case '/': *o++ = '/'; break;
        case 'b': *o++ = '\b'; break;
        case 'f': *o++ = '\f'; break;
        case 'n': *o++ = '\n'; break;
        case 'r': *o++ = '\r'; break;
        case 't': *o++ = '\t'; break;
        case 'u': {
            unsigned cp, lo;
            if (hex4(ps, p, &cp)) {
                ps->p = p;
                fail(ps, "invalid escape");
                free(out);
                return NULL;
            }
            p += 4;
            if (cp >= 0xD800 && cp <= 0xDBFF) { /* surrogate pair */
                if (p + 6 <= q && p[0] == '\\' && p[1] == 'u' && !hex4(ps, p + 2, &lo) &&
                    lo >= 0xDC00 && lo <= 0xDFFF) {
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    p += 6;
                } else {
                    ps->p = p;
                    fail(ps, "invalid Unicode '\\u%04X'", cp);
                    free(out);
                    return NULL;
                }
            } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
                ps->p = p;
                fail(ps, "invalid Unicode '\\u%04X'", cp);
                free(out);
                return NULL;
            }
            o = put_utf8(o, cp);
            break;
        }
        default:
            ps->p = p - 1;
            fail(ps, "invalid escape");
            free(out);
            return NULL;
        }
    }
    *o = '\0';
    *len = (size_t)(o - out);
    ps->p = q + 1;
    return out;
}

static int is_digit(parser *ps, const char *p)
{
    return p < ps->end && *p >= '0' && *p <= '9';
}

static json_t *parse_number(parser *ps)
{
    const char *p = ps->p, *st = p;
    int real = 0;
    if (*p == '-')
        p++;
    if (is_digit(ps, p) && *p == '0') {
        p++;
        if (is_digit(ps, p)) {
            fail(ps, "invalid token");
            return NULL;
        }
    } else if (is_digit(ps, p)) {
        while (is_digit(ps, p))
            p++;
    } else {
        fail(ps, "invalid token");
        return NULL;
    }
    if (p < ps->end && *p == '.') {
        real = 1;
        p++;
        if (!is_digit(ps, p)) {
            ps->p = p;
            fail(ps, "invalid token");
            return NULL;
        }
        while (is_digit(ps, p))
            p++;
    }
    if (p < ps->end && (*p == 'e' || *p == 'E')) {
        real = 1;
        p++;
        if (p < ps->end && (*p == '+' || *p == '-'))
            p++;
        if (!is_digit(ps, p)) {
            ps->p = p;
            fail(ps, "invalid token");
            return NULL;
        }
        while (is_digit(ps, p))
            p++;
    }
    const size_t n = (size_t)(p - st);
    char *buf = malloc(n + 1);
    if (!buf) {
        fail(ps, "out of memory");
        return NULL;
    }
    memcpy(buf, st, n);
    buf[n] = '\0';
    json_t *out = NULL;
    errno = 0;
    if (!real) {
        const long long v = strtoll(buf, NULL, 10);
        if (errno == ERANGE) {
            fail(ps, "too big %sinteger", v < 0 ? "negative " : "");
        } else if ((out = alloc_value(sizeof(jint), JSON_INTEGER))) {
            ((jint *)out)->v = v;
        }
    } else {
        const double v = strtod(buf, NULL);
        if (errno == ERANGE && (v == HUGE_VAL || v == -HUGE_VAL)) {
            fail(ps, "real number overflow");
        } else if ((out = alloc_value(sizeof(jreal), JSON_REAL))) {
            ((jreal *)out)->v = v;
        }
    }
    free(buf);
    if (!out && !ps->failed)
        fail(ps, "out of memory");
    ps->p = p;
    return out;
}

static json_t *parse_array(parser *ps, int depth);
static json_t *parse_object(parser *ps, int depth);

static int word(parser *ps, const char *w)
{
    const size_t n = strlen(w);
    if ((size_t)(ps->end - ps->p) >= n && !memcmp(ps->p, w, n)) {
        ps->p += n;
        return 1;
    }
    return 0;
}

static json_t *parse_value(parser *ps, int depth)
{
    skip_ws(ps);
    if (ps->p >= ps->end) {
        fail(ps, "unexpected end of input");
        return NULL;
    }
    if (depth > kMaxDepth) {
        fail(ps, "maximum parsing depth reached");
        return NULL;
    }
    switch (*ps->p) {
    case '{': return parse_object(ps, depth + 1);
    case '[': return parse_array(ps, depth + 1);
    case '"': {
        size_t len;
        char *s = parse_string_raw(ps, &len);
        if (!s)
            return NULL;
        json_t *j = alloc_value(sizeof(jstr), JSON_STRING);
        if (!j) {
            free(s);
            fail(ps, "out of memory");
            return NULL;
        }
        ((jstr *)j)->s = s;
        return j;
    }
    case 't':
        if (word(ps, "true")) return &s_true;
        break;
    case 'f':
        if (word(ps, "false")) return &s_false;
        break;
    case 'n':
        if (word(ps, "null")) return &s_null;
        break;
    default:
        if (*ps->p == '-' || (*ps->p >= '0' && *ps->p <= '9'))
            return parse_number(ps);
    }
    fail(ps, "invalid token");
    return NULL;
}

static json_t *parse_array(parser *ps, int depth)
{
    jarr *a = (jarr *)alloc_value(sizeof(jarr), JSON_ARRAY);
    if (!a) {
        fail(ps, "out of memory");
        return NULL;
    }
    ps->p++; /* '[' */
    skip_ws(ps);
    if (ps->p < ps->end && *ps->p == ']') {
        ps->p++;
        return &a->j;
    }
    for (;;) {
        json_t *v = parse_value(ps, depth);
        if (!v)
            goto bad;
        if (push((void ***)&a->v, &a->n, &a->cap, v)) {
            json_decref(v);
            fail(ps, "out of memory");
            goto bad;
        }
        skip_ws(ps);
        if (ps->p < ps->end && *ps->p == ',') {
            ps->p++;
            continue;
        }
        if (ps->p < ps->end && *ps->p == ']') {
            ps->p++;
            return &a->j;
        }
        fail(ps, "']' expected");
        goto bad;
    }
bad:
    json_delete(&a->j);
    return NULL;
}

static json_t *parse_object(parser *ps, int depth)
{
    jobj *o = (jobj *)alloc_value(sizeof(jobj), JSON_OBJECT);
    if (!o) {
        fail(ps, "out of memory");
        return NULL;
    }
    ps->p++; /* '{' */
    skip_ws(ps);
    if (ps->p < ps->end && *ps->p == '}') {
        ps->p++;
        return &o->j;
    }
    for (;;) {
        skip_ws(ps);
        if (ps->p >= ps->end || *ps->p != '"') {
            fail(ps, "string or '}' expected");
            goto bad;
        }
        size_t len;
        char *k = parse_string_raw(ps, &len);
        if (!k)
            goto bad;
        if (strlen(k) != len) {
            free(k);
            fail(ps, "NUL byte in object key not supported");
            goto bad;
        }
        skip_ws(ps);
        if (ps->p >= ps->end || *ps->p != ':') {
            free(k);
            fail(ps, "':' expected");
            goto bad;
        }
        ps->p++;
        json_t *v = parse_value(ps, depth);
        if (!v) {
            free(k);
            goto bad;
        }
        size_t i = 0;
        while (i < o->n && strcmp(o->k[i], k)) /* a repeated key: last one wins */
            i++;
        if (i < o->n) {
            free(k);
            json_decref(o->v[i]);
            o->v[i] = v;
        } else {
            size_t nk = o->n, ck = o->cap;
            if (push((void ***)&o->k, &nk, &ck, k) ||
                push((void ***)&o->v, &o->n, &o->cap, v)) {
                free(k);
                json_decref(v);
                fail(ps, "out of memory");
                goto bad;
            }
        }
        skip_ws(ps);
        if (ps->p < ps->end && *ps->p == ',') {
            ps->p++;
            continue;
        }
        if (ps->p < ps->end && *ps->p == '}') {
            ps->p++;
            return &o->j;
        }
        fail(ps, "'}' expected");
        goto bad;
    }
bad:
    json_delete(&o->j);
    return NULL;
}

static json_t *load_buffer(const char *s, size_t n, json_error_t *error)
{
    parser ps = {s, s, s + n, s, 1, error, 0};
    if (error) {
        memset(error, 0, sizeof(*error));
        strcpy(error->source, "<input>");
    }
    if (memchr(s, '\0', n)) {
        ps.p = (const char *)memchr(s, '\0', n);
        fail(&ps, "\\u0000 is not allowed without JSON_ALLOW_NUL");
        return NULL;
    }
    skip_ws(&ps);
    if (ps.p >= ps.end || (*ps.p != '[' && *ps.p != '{')) {
        fail(&ps, "'[' or '{' expected");
        return NULL;
    }
    json_t *root = parse_value(&ps, 0);
    if (!root)
        return NULL;
    skip_ws(&ps);
    if (ps.p != ps.end) {
        fail(&ps, "end of file expected");
        json_decref(root);
        return NULL;
    }
    return root;
}

json_t *json_loads(const char *input, size_t flags, json_error_t *error)
{
    (void)flags;
    if (!input) {
        if (error) {
            memset(error, 0, sizeof(*error));
            strcpy(error->text, "wrong arguments");
        }
        return NULL;
    }
    return load_buffer(input, strlen(input), error);
}

json_t *json_loadf(FILE *input, size_t flags, json_error_t *error)
{
    (void)flags;
    if (!input) {
        if (error) {
            memset(error, 0, sizeof(*error));
            strcpy(error->text, "wrong arguments");
        }
        return NULL;
    }
    size_t n = 0, cap = 1 << 16;
    char *buf = malloc(cap);
    while (buf) {
        n += fread(buf + n, 1, cap - n, input);
        if (n < cap)
            break;
        char *nb = realloc(buf, cap * 2);
        if (!nb) {
            free(buf);
            buf = NULL;
            break;
        }
        buf = nb;
        cap *= 2;
    }
    if (!buf) {
        if (error) {
            memset(error, 0, sizeof(*error));
            strcpy(error->text, "out of memory");
        }
        return NULL;
    }
    json_t *root = load_buffer(buf, n, error);
    free(buf);
    return root;
}

void json_delete(json_t *json)
{
    if (!json || json->refcount == (size_t)-1)
        return;
    switch (json->type) {
    case JSON_ARRAY: {
        jarr *a = (jarr *)json;
        for (size_t i = 0; i < a->n; ++i)
            json_decref(a->v[i]);
        free(a->v);
        break;
    }
    case JSON_OBJECT: {
        jobj *o = (jobj *)json;
        for (size_t i = 0; i < o->n; ++i) {
            free(o->k[i]);
            json_decref(o->v[i]);
        }
        free(o->k);
        free(o->v);
        break;
    }
    case JSON_STRING:
        free(((jstr *)json)->s);
        break;
    default:
        break;
    }
    free(json);
}

size_t json_array_size(const json_t *array)
{
    return json_is_array(array) ? ((const jarr *)array)->n : 0;
}

json_t *json_array_get(const json_t *array, size_t index)
{
    if (!json_is_array(array) || index >= ((const jarr *)array)->n)
        return NULL;
    return ((const jarr *)array)->v[index];
}

json_t *json_object_get(const json_t *object, const char *key)
{
    if (!json_is_object(object) || !key)
        return NULL;
    const jobj *o = (const jobj *)object;
    for (size_t i = 0; i < o->n; ++i)
        if (!strcmp(o->k[i], key))
            return o->v[i];
    return NULL;
}

json_int_t json_integer_value(const json_t *integer)
{
    return json_is_integer(integer) ? ((const jint *)integer)->v : 0;
}

double json_real_value(const json_t *real)
{
    return json_is_real(real) ? ((const jreal *)real)->v : 0.0;
}

const char *json_string_value(const json_t *string)
{
    return json_is_string(string) ? ((const jstr *)string)->s : NULL;
}

// formats.cpp -- the reference's on-disk record formats on the hot path's two edges
// (SURVEY.md §8(f) #3): host code, no device work.
//
//   * point text  -> n x d FP64   MapperDataset_github.call (MapperDataset_github.java:12-20):
//                                  s.split(" ") + Double.parseDouble per field, one point per
//                                  line.  strict = 1 keeps exactly that (a doubled space is an
//                                  empty field -> NumberFormatException); strict = 0 is
//                                  deviation D1 (any run of blanks/tabs separates fields, the
//                                  first d fields are kept: Skin_NonSkin is TAB-separated with
//                                  a label column).
//   * local-MST records <-> text  CreateLocalMST.java:110-123 writes "v1 v2 w f1 f2 node"
//                                  lines joined by '\n' (no trailing newline), w via
//                                  Double.toString; UnionFindReducer.java:22-45 reads them back
//                                  with split("\n"), split(" "), Integer.parseInt and
//                                  Double.parseDouble.
//
// Double.toString: Java's layout rules (plain for 1e-3 <= |v| < 1e7, else d.dddE<exp>; at
// least one fractional digit) with the shortest digit string that parses back to the same
// double (the closest such; when one digit suffices, the closest of length <= 2) -- the
// JDK >= 19 digits.  JDK 8's FloatingDecimal emits a
// longer string for a few rare values (JDK-4511638); both parse back to the same bits.
#include <algorithm>
#include <clocale>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <locale.h>
#include <string>
#include <vector>

#include "internal.hpp"

namespace hdb {

namespace {

int fail(int code, const char *fmt, ...) {
    char msg[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    set_error(msg);
    return code;
}

locale_t c_locale() {
    static locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    return loc;
}

bool is_digit(char c) { return c >= '0' && c <= '9'; }
bool is_hex(char c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

// Double.parseDouble (FloatingDecimal.readJavaFormatString): trim chars <= ' ', optional
// sign, then "NaN" | "Infinity" | decimal [eE exp] | hex 0x..p exp, optional [fFdD] suffix.
// Returns false where Java throws NumberFormatException.
bool java_parse_double(const char *b, const char *e, double *out) {
    while (b < e && (unsigned char)*b <= ' ') ++b;
    while (e > b && (unsigned char)e[-1] <= ' ') --e;
    if (b == e) return false;
    const char *p = b;
    bool neg = false;
    if (*p == '+' || *p == '-') neg = *p++ == '-';
    size_t rest = (size_t)(e - p);
    if (rest == 3 && !memcmp(p, "NaN", 3)) {
        *out = __builtin_nan("");
        return true;
    }
    if (rest == 8 && !memcmp(p, "Infinity", 8)) {
        *out = neg ? -__builtin_inf() : __builtin_inf();
        return true;
    }
    const char *q = p;
    if (rest >= 2 && q[0] == '0' && (q[1] == 'x' || q[1] == 'X')) {
        q += 2;
        int nd = 0;
        while (q < e && is_hex(*q)) ++q, ++nd;
        if (q < e && *q == '.') {
            ++q;
            while (q < e && is_hex(*q)) ++q, ++nd;
        }
        if (nd == 0 || q >= e || (*q != 'p' && *q != 'P')) return false;
        ++q;
    } else {
        int nd = 0;
        while (q < e && is_digit(*q)) ++q, ++nd;
        if (q < e && *q == '.') {
            ++q;
            while (q < e && is_digit(*q)) ++q, ++nd;
        }
        if (nd == 0) return false;
        if (q < e && (*q == 'e' || *q == 'E')) {
            ++q;
        } else {
            goto suffix;
        }
    }
    // exponent digits (mandatory after e/E/p/P)
    {
        if (q < e && (*q == '+' || *q == '-')) ++q;
        int ne = 0;
        while (q < e && is_digit(*q)) ++q, ++ne;
        if (ne == 0) return false;
    }
suffix:
    const char *num_end = q;
    if (q < e && (*q == 'f' || *q == 'F' || *q == 'd' || *q == 'D')) ++q;
    if (q != e) return false;
    std::string s(b, num_end);
    // a type suffix (f/F/d/D) does not influence the result of Double.parseDouble (its
    // javadoc; FloatingDecimal returns the same digits' doubleValue)
    *out = strtod_l(s.c_str(), nullptr, c_locale());
    return true;
}

// Integer.parseInt(s) (radix 10): optional sign, >= 1 digit, no whitespace, int range.
bool java_parse_int(const char *b, const char *e, int32_t *out) {
    if (b == e) return false;
    bool neg = false;
    if (*b == '+' || *b == '-') {
        neg = *b++ == '-';
        if (b == e) return false;
    }
    int64_t v = 0;
    for (; b < e; ++b) {
        if (!is_digit(*b)) return false;
        v = v * 10 + (*b - '0');
        if (v > (int64_t)INT32_MAX + 1) return false;
    }
    if (neg) v = -v;
    if (v > INT32_MAX || v < INT32_MIN) return false;
    *out = (int32_t)v;
    return true;
}

// String.split(String) with a one-char literal: no separator -> the whole string (even
// ""); otherwise every separator splits, trailing empty strings are removed and a leading
// empty string is kept.
void java_split(const char *b, const char *e, char sep, std::vector<std::pair<const char *, const char *>> &f) {
    f.clear();
    const char *s = b;
    for (const char *p = b; p < e; ++p)
        if (*p == sep) {
            f.emplace_back(s, p);
            s = p + 1;
        }
    f.emplace_back(s, e);
    if (f.size() == 1) return;
    while (!f.empty() && f.back().first == f.back().second) f.pop_back();
}

}  // namespace

// Double.toString digits + layout; returns the string length (< 32).
int java_double_to_string(double v, char *buf) {
    if (v != v) return (int)(strcpy(buf, "NaN"), 3);
    if (v == __builtin_inf()) return (int)(strcpy(buf, "Infinity"), 8);
    if (v == -__builtin_inf()) return (int)(strcpy(buf, "-Infinity"), 9);
    char *o = buf;
    if (std::signbit(v)) *o++ = '-', v = -v;
    if (v == 0.0) {
        strcpy(o, "0.0");
        return (int)(o - buf) + 3;
    }
    // shortest p in [1, 17] with a p-digit decimal that parses back to v.  The nearest
    // p-digit decimal (%.*e) is the candidate; at a power of two the rounding interval is
    // asymmetric (the lower gap is half the upper), so when the nearest one misses, the
    // next p-digit decimal upwards (the wider side) can still be inside: try it too.
    char tmp[40];
    auto fits = [&](int p, char *cand) {
        snprintf(cand, 40, "%.*e", p - 1, v);
        if (strtod_l(cand, nullptr, c_locale()) == v) return true;
        double m, x = v;
        int ex = 0;
        m = std::frexp(x, &ex);
        if (m != 0.5) return false;  // not a power of two: the interval is symmetric
        // bump the last digit of the nearest candidate by one unit
        char dg[24];
        int nd = 0;
        const char *t = cand;
        for (; *t && *t != 'e'; ++t)
            if (is_digit(*t)) dg[nd++] = *t;
        int E = atoi(t + 1);
        int i = nd - 1;
        while (i >= 0 && dg[i] == '9') dg[i--] = '0';
        if (i < 0) {  // 9.99 -> 10.0: one more leading digit
            dg[0] = '1';
            for (int j = 1; j < nd; ++j) dg[j] = '0';
            ++E;
        } else {
            ++dg[i];
        }
        char up[40], *o = up;
        *o++ = dg[0];
        if (nd > 1) {
            *o++ = '.';
            for (int j = 1; j < nd; ++j) *o++ = dg[j];
        }
        sprintf(o, "e%d", E);
        if (strtod_l(up, nullptr, c_locale()) != v) return false;
        strcpy(cand, up);
        return true;
    };
    int lo = 1;
    while (lo < 17 && !fits(lo, tmp)) ++lo;
    // Java's rule when one digit suffices: the closest decimal of length 1 or 2, i.e. the
    // correctly rounded 2-digit one (4.9E-324, not 5.0E-324)
    if (lo < 2) lo = 2;
    if (!fits(lo, tmp)) snprintf(tmp, sizeof tmp, "%.*e", lo - 1, v);
    char dig[20];
    int nd = 0;
    const char *t = tmp;
    for (; *t && *t != 'e'; ++t)
        if (is_digit(*t)) dig[nd++] = *t;
    int E = atoi(t + 1);
    while (nd > 1 && dig[nd - 1] == '0') --nd;  // trailing zeros carry no digits
    if (E >= -3 && E <= 6) {                      // plain: 1e-3 <= v < 1e7
        if (E >= 0) {
            for (int i = 0; i <= E; ++i) *o++ = i < nd ? dig[i] : '0';
            *o++ = '.';
            if (nd > E + 1)
                for (int i = E + 1; i < nd; ++i) *o++ = dig[i];
            else
                *o++ = '0';
        } else {
            *o++ = '0';
            *o++ = '.';
            for (int i = 0; i < -E - 1; ++i) *o++ = '0';
            for (int i = 0; i < nd; ++i) *o++ = dig[i];
        }
    } else {
        *o++ = dig[0];
        *o++ = '.';
        if (nd > 1)
            for (int i = 1; i < nd; ++i) *o++ = dig[i];
        else
            *o++ = '0';
        o += sprintf(o, "E%d", E);
    }
    *o = 0;
    return (int)(o - buf);
}

}  // namespace hdb

using namespace hdb;

extern "C" {

int hdb_format_double(double v, char *buf, int32_t cap) {
    char tmp[40];
    int n = java_double_to_string(v, tmp);
    if (!buf || cap <= n) return fail(HDB_EINVAL, "hdb_format_double: buffer needs %d bytes", n + 1);
    memcpy(buf, tmp, (size_t)n + 1);
    return n;
}

int hdb_parse_points(const char *text, int64_t len, int32_t d, int32_t strict, double *X, int64_t cap,
                     int64_t *n_out, int32_t *d_out) {
    if (!text || len < 0 || !n_out || d < 0) return fail(HDB_EINVAL, "hdb_parse_points: bad arguments");
    if (X && cap < 0) return fail(HDB_EINVAL, "hdb_parse_points: negative capacity");
    const char *p = text, *end = text + len;
    std::vector<std::pair<const char *, const char *>> f;
    std::vector<double> row;
    int64_t n = 0, line_no = 0;
    int32_t dd = d;
    while (p < end) {
        const char *le = (const char *)memchr(p, '\n', (size_t)(end - p));
        if (!le) le = end;
        const char *lb = p, *lend = le;
        p = le + 1;
        ++line_no;
        if (lend > lb && lend[-1] == '\r') --lend;  // BufferedReader.readLine drops CR too
        f.clear();
        if (strict) {
            java_split(lb, lend, ' ', f);  // an empty line is [""] -> parseDouble("") throws
        } else {
            const char *q = lb;
            while (q < lend) {
                while (q < lend && (*q == ' ' || *q == '\t')) ++q;
                if (q >= lend) break;
                const char *s = q;
                while (q < lend && *q != ' ' && *q != '\t') ++q;
                f.emplace_back(s, q);
            }
            if (f.empty()) continue;  // D1: blank lines carry no point
        }
        if (dd == 0) dd = (int32_t)f.size();
        // the Java parses every field of the line before anything checks the count
        const int32_t np = strict ? (int32_t)f.size() : std::min<int32_t>((int32_t)f.size(), dd);
        row.resize((size_t)np);
        for (int32_t j = 0; j < np; ++j)
            if (!java_parse_double(f[j].first, f[j].second, &row[j]))
                return fail(HDB_EREF_NUMBER_FORMAT, "hdb_parse_points: For input string: \"%.*s\" (line %lld)",
                            (int)(f[j].second - f[j].first), f[j].first, (long long)line_no);
        if (np < dd || (strict && np != dd))
            return fail(HDB_EREF_OOB, "hdb_parse_points: line %lld has %zu fields, expected %d",
                        (long long)line_no, f.size(), dd);
        if (X && n >= cap) return fail(HDB_EINVAL, "hdb_parse_points: more than %lld points", (long long)cap);
        if (X) memcpy(X + n * dd, row.data(), sizeof(double) * (size_t)dd);
        ++n;
    }
    *n_out = n;
    if (d_out) *d_out = dd;
    return HDB_OK;
}

int hdb_format_mst_records(const int32_t *va, const int32_t *vb, const double *w, const int32_t *fake1,
                           const int32_t *fake2, const int32_t *node, int64_t ne, char *out, int64_t cap,
                           int64_t *len_out) {
    if ((ne > 0 && (!va || !vb || !w)) || ne < 0 || !len_out)
        return fail(HDB_EINVAL, "hdb_format_mst_records: bad arguments");
    int64_t len = 0;
    char line[160];
    for (int64_t i = 0; i < ne; ++i) {
        char ws[40];
        java_double_to_string(w[i], ws);
        int k = snprintf(line, sizeof line, "%s%d %d %s %d %d %d", i ? "\n" : "", va[i], vb[i], ws,
                         fake1 ? fake1[i] : 0, fake2 ? fake2[i] : 0, node ? node[i] : 0);
        if (out) {
            if (len + k >= cap) return fail(HDB_EINVAL, "hdb_format_mst_records: output buffer too small");
            memcpy(out + len, line, (size_t)k);
        }
        len += k;
    }
    if (out) {
        if (len >= cap) return fail(HDB_EINVAL, "hdb_format_mst_records: output buffer too small");
        out[len] = 0;
    }
    *len_out = len;
    return HDB_OK;
}

int hdb_parse_mst_records(const char *text, int64_t len, int32_t *va, int32_t *vb, double *w, int32_t *fake1,
                          int32_t *fake2, int32_t *node, int64_t cap, int64_t *ne_out) {
    if (!text || len < 0 || !ne_out) return fail(HDB_EINVAL, "hdb_parse_mst_records: bad arguments");
    std::vector<std::pair<const char *, const char *>> lines, f;
    java_split(text, text + len, '\n', lines);
    const bool fill = va != nullptr;
    if (fill && (int64_t)lines.size() > cap)
        return fail(HDB_EINVAL, "hdb_parse_mst_records: %zu records exceed capacity %lld", lines.size(),
                    (long long)cap);
    int64_t i = 0;
    for (auto &ln : lines) {
        java_split(ln.first, ln.second, ' ', f);
        // UnionFindReducer.java:26-31 reads data[0] .. data[5] in order: a bad early field
        // throws NumberFormatException before a missing later index throws
        // ArrayIndexOutOfBoundsException
        int32_t iv[6] = {0, 0, 0, 0, 0, 0};
        double ww = 0.0;
        for (size_t k = 0; k < 6; ++k) {
            if (k >= f.size())
                return fail(HDB_EREF_OOB, "hdb_parse_mst_records: record %lld has %zu fields", (long long)i, f.size());
            const bool ok = k == 2 ? java_parse_double(f[k].first, f[k].second, &ww)
                                   : java_parse_int(f[k].first, f[k].second, &iv[k]);
            if (!ok)
                return fail(HDB_EREF_NUMBER_FORMAT, "hdb_parse_mst_records: record %lld: For input string: \"%.*s\"",
                            (long long)i, (int)(f[k].second - f[k].first), f[k].first);
        }
        const int32_t a = iv[0], b = iv[1], f1 = iv[3], f2 = iv[4], nd = iv[5];
        if (fill) {
            va[i] = a, vb[i] = b, w[i] = ww;
            if (fake1) fake1[i] = f1;
            if (fake2) fake2[i] = f2;
            if (node) node[i] = nd;
        }
        ++i;
    }
    *ne_out = i;
    return HDB_OK;
}

}  // extern "C"

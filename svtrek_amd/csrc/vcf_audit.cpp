// vcf_audit.cpp -- VCF record parsing (A1) and refined-call printing (A11) for the
// `svtrek audt` drop-in.  Behaviour follows the reference byte for byte:
//   parse:  thread_func, reference audit.c:62-173 (strtok_r tokenisation, strstr
//           "SVTYPE=" / "END=" -- the latter also matching inside "CIEND=" --, strtol
//           into uint32, the length inference when SVTYPE is absent, the 50-bp filter);
//   print:  audit.c:176-232 printf formats (%u / %d of uint32 values, NA for 0xFFFFFFFF).
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "svtrek_host.h"

namespace {

constexpr int SV_MIN_LENGTH = 50;   // params.h:33

int sv_type_of(const char *s) {     // parse_sv_type, audit.c:3-11
    if (!strcmp(s, "INS") || !strcmp(s, "INS:ME")) return SVT_INS;
    if (!strcmp(s, "DEL") || !strcmp(s, "DEL:ME")) return SVT_DEL;
    if (!strcmp(s, "INV")) return SVT_INV;
    if (!strcmp(s, "DUP")) return SVT_DUP;
    if (!strcmp(s, "TRA")) return SVT_TRA;
    if (!strcmp(s, "BND")) return SVT_BND;
    return SVT_UNKNOWN;
}

// copy the value after `key` up to ';' (at most cap-1 bytes), as audit.c:119-129 / :148-158
void info_value(const char *v, char *buf, size_t cap) {
    const char *e = strchr(v, ';');
    size_t len = e ? (size_t)(e - v) : strlen(v);
    if (len >= cap) len = cap - 1;
    memcpy(buf, v, len);
    buf[len] = 0;
}

// [b, e) of the text split into `parts` pieces that start right after a '\n'
std::vector<size_t> line_cuts(const char *text, size_t len, int parts) {
    std::vector<size_t> cut{0};
    for (int t = 1; t < parts; t++) {
        size_t c = len * (size_t)t / (size_t)parts;
        const void *nl = c < len ? memchr(text + c, '\n', len - c) : nullptr;
        c = nl ? (size_t)((const char *)nl - text) + 1 : len;
        cut.push_back(std::max(c, cut.back()));
    }
    cut.push_back(len);
    return cut;
}

template <typename F>
void run_parts(int parts, F &&f) {
    if (parts <= 1) { f(0); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < parts; t++) th.emplace_back([&, t] { f(t); });
    for (auto &x : th) x.join();
}

}  // namespace

struct svth_vcf {
    std::vector<svt_locus> loci;
    std::string msgs;
};

extern "C" {

// One logical VCF line of process_vcf's reader (audit.c:299-327) -> o.
static void vcf_take(char *line, svth_vcf &o, char *perr, size_t cap) {
    svt_locus l;
    const int act = svth_parse_line(line, &l, perr, cap);
    if (act == 2) o.msgs += perr;
    if (act != 1) return;
    if (svth_is_unknown_type(&l)) o.msgs += "[ERROR] Unkown type.\n";
    o.loci.push_back(l);
}

// The reader loop of audit.c:294-327 exactly, sequentially: fgets into a buffer of current_size
// bytes (1 MiB, doubled whenever a line fills it, never shrunk), strlen (a line ends at its
// first NUL; the rest of what that fgets read is dropped), a final line without '\n' that exactly
// fills the buffer skipped (the next fgets returns NULL, :317), lines shorter than 2 chars and
// '#' lines skipped.  Used when the file has a line of 1 MiB or more (the buffer's history
// matters then); svth_vcf_parse's threaded loop is the same for every shorter line.
static void vcf_parse_exact(const char *text, size_t len, svth_vcf &o) {
    size_t cur = 1u << 20, pos = 0;
    std::string buf(cur, '\0');
    char perr[1024];
    // fgets(buf + at, cap): up to cap - 1 chars through the first '\n'; false (NULL) at the end
    auto fgets_at = [&](size_t at, size_t cap) {
        if (pos >= len) return false;
        const size_t room = std::min(cap - 1, len - pos);
        const void *nl = memchr(text + pos, '\n', room);
        const size_t k = nl ? (size_t)((const char *)nl - (text + pos)) + 1 : room;
        memcpy(&buf[at], text + pos, k);
        buf[at + k] = '\0';
        pos += k;
        return true;
    };
    while (fgets_at(0, cur)) {
        size_t n = strlen(buf.c_str());
        bool skip = false;
        while (n == cur - 1 && buf[n - 1] != '\n') {   // audit.c:304-319
            cur *= 2;
            buf.resize(cur);
            if (!fgets_at(n, cur - n)) { skip = true; break; }
            n = strlen(buf.c_str());
        }
        if (skip || n < 2 || buf[0] == '#') continue;   // :321-322
        if (buf[n - 1] == '\n') n--;                     // :324-327
        std::string line(buf.data(), n);
        vcf_take(&line[0], o, perr, sizeof perr);
    }
}

svth_vcf *svth_vcf_parse(const char *text, size_t len, int threads) {
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), len / (1u << 20) + 1));
    const std::vector<size_t> cut = line_cuts(text, len, T);
    std::vector<svth_vcf> part((size_t)T);
    std::atomic<bool> long_line{false};
    run_parts(T, [&](int t) {
        svth_vcf &o = part[(size_t)t];
        std::string line;
        char perr[1024];
        for (size_t i = cut[(size_t)t], e = cut[(size_t)t + 1]; i < e;) {
            const void *nl = memchr(text + i, '\n', e - i);
            const size_t n = (nl ? (size_t)((const char *)nl - text) + 1 : e) - i;
            const char *ln = text + i;
            i += n;
            // a physical line of 1 MiB - 1 chars or more: the reader's buffer history decides
            // (vcf_parse_exact); shorter ones are one fgets each
            if (n >= (1u << 20) - 1) { long_line = true; return; }
            const void *z = memchr(ln, '\0', n);               // strlen: the line ends at a NUL
            const size_t m = z ? (size_t)((const char *)z - ln) : n;
            if (m < 2 || ln[0] == '#') continue;                     // audit.c:321-322
            line.assign(ln, ln[m - 1] == '\n' ? m - 1 : m);         // :324-327
            vcf_take(&line[0], o, perr, sizeof perr);
        }
    });
    svth_vcf *v = new svth_vcf();
    if (long_line) {
        vcf_parse_exact(text, len, *v);
        return v;
    }
    size_t n = 0;
    for (auto &p : part) n += p.loci.size();
    v->loci.reserve(n);
    for (auto &p : part) {
        v->loci.insert(v->loci.end(), p.loci.begin(), p.loci.end());
        v->msgs += p.msgs;
    }
    return v;
}

size_t svth_vcf_count(const svth_vcf *v) { return v->loci.size(); }
const svt_locus *svth_vcf_loci(const svth_vcf *v) { return v->loci.data(); }
const char *svth_vcf_messages(const svth_vcf *v, size_t *len) {
    if (len) *len = v->msgs.size();
    return v->msgs.c_str();
}
void svth_vcf_free(svth_vcf *v) { delete v; }

char *svth_format_batch(const svt_locus *l, const svt_result *r, size_t n, int threads, size_t *len) {
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), n / 16384 + 1));
    std::vector<std::string> part((size_t)T);
    run_parts(T, [&](int t) {
        std::string &o = part[(size_t)t];
        const size_t b = n * (size_t)t / (size_t)T, e = n * (size_t)(t + 1) / (size_t)T;
        o.reserve((e - b) * 128);
        char buf[512];
        for (size_t k = b; k < e; k++) {
            const int m = svth_format(&l[k], &r[k], buf, sizeof buf);
            if (m > 0) o.append(buf, (size_t)m);
        }
    });
    size_t tot = 0;
    for (auto &p : part) tot += p.size();
    char *out = (char *)malloc(tot + 1);
    if (!out) return nullptr;
    size_t at = 0;
    for (auto &p : part) { memcpy(out + at, p.data(), p.size()); at += p.size(); }
    out[tot] = 0;
    if (len) *len = tot;
    return out;
}

void svth_free(void *p) { free(p); }

int svth_parse_line(char *line, svt_locus *l, char *err, size_t errcap) {
    char *save = nullptr, *alt_save = nullptr;
    if (err && errcap) err[0] = 0;
    char *chrom = strtok_r(line, "\t", &save);
    char *index = strtok_r(nullptr, "\t", &save);
    if (!index) {
        if (err) snprintf(err, errcap, "VCF: no index at line: %s\n", line);
        return 2;
    }
    strtok_r(nullptr, "\t", &save);                       // ID
    char *seq = strtok_r(nullptr, "\t", &save);           // REF
    char *alt = seq ? strtok_r(nullptr, "\t", &save) : nullptr;
    if (!seq || !alt) {   // the reference dereferences NULL here; report and skip instead
        if (err) snprintf(err, errcap, "VCF: truncated record at POS %s\n", index);
        return 2;
    }
    size_t seq_len = strlen(seq), max_alt = 0, min_alt = 0x7FFFFFFF;
    for (char *t = strtok_r(alt, ",", &alt_save); t; t = strtok_r(nullptr, ",", &alt_save)) {
        size_t k = strlen(t);
        if (k > max_alt) max_alt = k;
        if (k < min_alt) min_alt = k;
    }
    strtok_r(nullptr, "\t", &save);                       // QUAL
    strtok_r(nullptr, "\t", &save);                       // FILTER
    char *info = strtok_r(nullptr, "\t", &save);          // INFO
    if (!info) {
        if (err) snprintf(err, errcap, "VCF: truncated record at POS %s\n", index);
        return 2;
    }
    int chrom_index = strncmp(chrom, "chr", 3) == 0 ? atoi(chrom + 3) : atoi(chrom);
    uint32_t pos = (uint32_t)strtol(index, nullptr, 10);
    if (pos == 0 && index[0] != '0') {
        if (err) snprintf(err, errcap, "[ERROR] Conversion error to pos %s\n", index);
        return 2;
    }
    int type;
    if (const char *sv = strstr(info, "SVTYPE=")) {
        char b[16];
        info_value(sv + 7, b, sizeof b);
        type = sv_type_of(b);
    } else if (seq_len == 1 && (size_t)SV_MIN_LENGTH < max_alt) {
        type = SVT_INS;
    } else if ((size_t)SV_MIN_LENGTH < seq_len && min_alt == 1) {
        type = SVT_DEL;
    } else {
        return 0;
    }
    uint32_t end;
    if (const char *es = strstr(info, "END=")) {
        char b[32];
        info_value(es + 4, b, sizeof b);
        end = (uint32_t)strtol(b, nullptr, 10);
        if (end == 0 && b[0] != '0') return 0;
    } else {
        end = pos + (uint32_t)seq_len;
    }
    if ((type == SVT_DEL || type == SVT_INV) && end - pos < (uint32_t)SV_MIN_LENGTH) return 0;
    l->type = type;
    l->chrom = chrom_index;
    l->pos = pos;
    l->end = end;
    return 1;
}

int svth_is_unknown_type(const svt_locus *l) {
    return !(l->type == SVT_INS || l->type == SVT_DEL || l->type == SVT_INV);
}

int svth_format(const svt_locus *l, const svt_result *r, char *buf, size_t cap) {
    const uint32_t pos = l->pos, end = l->end;
    buf[0] = 0;
    if (l->type == SVT_INS) {
        if (r->start == SVT_NA)
            return snprintf(buf, cap, "(INS) chr: %d, org pos: %u, ref pos: NA\n", l->chrom, pos);
        return snprintf(buf, cap, "(INS) chr: %d, org pos: %u, ref pos: %u, diff: %d\n", l->chrom, pos, r->start,
                        (int)(r->start - pos));
    }
    if (l->type == SVT_DEL) {
        if (!((uint32_t)SV_MIN_LENGTH < end - pos)) return 0;
        int n = snprintf(buf, cap, "(DEL) chr: %d, org pos: %u, org end: %u, ref pos: ", l->chrom, pos, end);
        auto put = [&](const char *fmt, long v) { n += snprintf(buf + n, cap - (size_t)n, fmt, v); };
        if (r->start == SVT_NA) n += snprintf(buf + n, cap - (size_t)n, "NA, ref end: ");
        else put("%ld, ref end: ", (long)(int)r->start);
        if (r->end == SVT_NA) n += snprintf(buf + n, cap - (size_t)n, "NA, ");
        else put("%ld, ", (long)(int)r->end);
        if (r->start == SVT_NA) n += snprintf(buf + n, cap - (size_t)n, "diff pos: NA, ");
        else put("diff pos: %ld, ", (long)(int)(r->start - pos));
        if (r->end == SVT_NA) n += snprintf(buf + n, cap - (size_t)n, "diff end: NA\n");
        else put("diff end: %ld\n", (long)(int)(r->end - end));
        return n;
    }
    if (l->type == SVT_INV) {
        if (!((uint32_t)SV_MIN_LENGTH < end - pos)) return 0;
        return snprintf(buf, cap, "(INV) chr: %d, org pos: %u, org end: %u, ref pos: %u, ref end: %u\n", l->chrom,
                        pos, end, r->start, r->end);
    }
    return 0;
}

}  // extern "C"

// svtrek_main.cpp -- `svtrek audt -b BAM -v VCF [OPTIONS]`, drop-in for the reference CLI
// (svtrek.c:5-22, init.c:21-147, audit.c:250-368) on MI355X.
//
// Same flags, defaults and stdout bytes as the reference; records are printed in VCF
// order (the reference prints in worker completion order and drops up to 2*T trailing
// records through its exit_signal race, SURVEY.md §3.1 -- not reproduced).  The work
// between the two [INFO] lines is: read the BAM once into a columnar pileup (host,
// -t inflate threads), copy it to HBM, parse all VCF records (A1), refine them in
// batched HIP launches (svt_refine_batch; --gpus N puts the records in genomic order,
// gives device g the g-th contiguous slice and uploads only the reads that slice's
// queries can reach; one host thread and one svt_ctx per device),
// print (A11).
#include <getopt.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <numeric>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <string>
#include <thread>
#include <vector>

#include "svtrek_gpu.h"
#include "svtrek_host.h"

namespace {

// params.h:27-36
constexpr int WIDER = 20000, MEDIAN = 10000, NARROW = 2000, CI_RANGE = 500, CI = 5, MIN_COUNT = 3, THREADS = 4;

void usage() {
    printf("Usage: ./svtrek [MODE] [OPTIONS]\n");
    printf("Mode:\n");
    printf("    disc    Variation discovery on graph alignment result.\n");
    printf("    audt    Audit the reported variations on VCF using BAM.\n");
}

void audt_usage() {
    printf("Usage: ./svtrek audt [-b|--bam BAM] [-v|--vcf VCF file] [OPTIONS]\n");
    printf("Options:\n");
    printf("    [-o|--ouput] <filename>           Output filename [Default: svtrek.out]\n");
    printf("    -t <num>                          Thread number [Default: %d]\n", THREADS);
    printf("    --verbose                         Verbose [Default: false]\n\n");
    printf("    --wider-interval <num>            Interval for the offset of the reads to start [Default: %d]\n", WIDER);
    printf("    --median-interval <num>           Interval for the offset of the reads (for point) [Default: %d]\n", MEDIAN);
    printf("    --narrow-interval <num>           Interval for the offset of the reads to end [Default: %d]\n", NARROW);
    printf("    --consensus-interval-range <num>  The interval to limit refinement range [DEFAULT: %d]\n", CI_RANGE);
    printf("    --consensus-interval <num>        The interval that is considered into the same position [DEFAULT: %d]\n", CI);
    printf("    --consensus-min-count <num>       Minimum number of elements needs for the consensus [Default: %d]\n\n", MIN_COUNT);
    printf("GPU options (svtrek_amd):\n");
    printf("    --gpus <num>                      GPUs to shard records over [Default: 1]\n");
    printf("    --device <num>                    First GPU index [Default: 0]\n");
    printf("    --devices <i,j,...>               Explicit GPU per shard (overrides --gpus/--device)\n");
    printf("    --batch <num>                     Records per GPU launch [Default: 1048576]\n");
    printf("    --spill-bytes <num>               Initial candidate spill pool per GPU; grown on demand [Default: 67108864]\n");
    printf("    --inflate <auto|gpu|cpu>          BGZF decompression of the BAM: first GPU or -t host threads;\n");
    printf("                                      auto: the GPU from 1 GiB of BAM on [Default: auto]\n");
}

struct Args {
    const char *bam = nullptr, *vcf = nullptr, *out = "svtrek.out";
    int threads = THREADS, verbose = 0, gpus = 1, device = 0, gpu_inflate = -1;   // -1: by BAM size
    size_t batch = 1u << 20;
    std::vector<int> devices;   // device of shard g
    svt_params prm{WIDER, MEDIAN, NARROW, CI_RANGE, CI, MIN_COUNT, 0};
};

void validate_file(const char *f, const char *msg) {   // init.c:35-47 (without its fclose(NULL) crash)
    if (!f) {
        fprintf(stderr, "%s\n", msg);
        exit(EXIT_FAILURE);
    }
    FILE *fp = fopen(f, "r");
    if (!fp) {
        fprintf(stderr, "[ERROR]: File couldn't be opened %s\n", f);
        exit(EXIT_FAILURE);
    }
    fclose(fp);
}

Args parse_audt(int argc, char **argv) {
    Args a;
    if (argc < 2) {
        audt_usage();
        exit(1);
    }
    static const option opts[] = {
        {"bam", required_argument, nullptr, 1}, {"vcf", required_argument, nullptr, 2},
        {"output", required_argument, nullptr, 3}, {"verbose", no_argument, nullptr, 4},
        {"wider-interval", required_argument, nullptr, 5}, {"median-interval", required_argument, nullptr, 6},
        {"narrow-interval", required_argument, nullptr, 7},
        {"consensus-interval-range", required_argument, nullptr, 8},
        {"consensus-interval", required_argument, nullptr, 9},
        {"consensus-min-count", required_argument, nullptr, 10}, {"help", no_argument, nullptr, 11},
        {"gpus", required_argument, nullptr, 20}, {"device", required_argument, nullptr, 21},
        {"batch", required_argument, nullptr, 22}, {"devices", required_argument, nullptr, 23},
        {"spill-bytes", required_argument, nullptr, 24}, {"inflate", required_argument, nullptr, 25},
        {nullptr, 0, nullptr, 0}};
    int opt, li;
    while ((opt = getopt_long(argc, argv, "b:v:o:t:h", opts, &li)) != -1) {
        switch (opt) {
        case 'b': case 1: a.bam = optarg; break;
        case 'v': case 2: a.vcf = optarg; break;
        case 'o': case 3: a.out = optarg; break;   // parsed, unused (as in the reference)
        case 4: a.verbose = 1; break;
        case 't': a.threads = atoi(optarg); break;
        case 5: a.prm.wider_interval = atoi(optarg); break;
        case 6: a.prm.median_interval = atoi(optarg); break;
        case 7: a.prm.narrow_interval = atoi(optarg); break;
        case 8: a.prm.consensus_interval_range = atoi(optarg); break;
        case 9: a.prm.consensus_interval = atoi(optarg); break;
        case 10: a.prm.consensus_min_count = atoi(optarg); break;
        case 'h': case 11: audt_usage(); exit(EXIT_SUCCESS);
        case 20: a.gpus = atoi(optarg); break;
        case 21: a.device = atoi(optarg); break;
        case 22: a.batch = (size_t)strtoull(optarg, nullptr, 10); break;
        case 24: a.prm.spill_bytes = (uint64_t)strtoull(optarg, nullptr, 10); break;
        case 25:
            if (strcmp(optarg, "gpu") && strcmp(optarg, "cpu") && strcmp(optarg, "auto")) {
                fprintf(stderr, "[ERROR] --inflate expects auto, gpu or cpu\n");
                exit(EXIT_FAILURE);
            }
            a.gpu_inflate = strcmp(optarg, "gpu") == 0 ? 1 : strcmp(optarg, "cpu") == 0 ? 0 : -1;
            break;
        case 23: {
            a.devices.clear();
            for (const char *p = optarg; *p;) {
                char *e;
                long d = strtol(p, &e, 10);
                if (e == p || d < 0) { fprintf(stderr, "[ERROR] --devices expects a list like 0,1,2\n"); exit(EXIT_FAILURE); }
                a.devices.push_back((int)d);
                p = *e == ',' ? e + 1 : e;
                if (*e && *e != ',') { fprintf(stderr, "[ERROR] --devices expects a list like 0,1,2\n"); exit(EXIT_FAILURE); }
            }
            break;
        }
        default:
            printf("[ERROR] Option %d is invalid.\n", opt);
            audt_usage();
            exit(EXIT_FAILURE);
        }
    }
    validate_file(a.bam, "[ERROR] BAM file is not provided.");
    validate_file(a.vcf, "[ERROR] VCF file is not provided.");
    // The reference deadlocks on -t 0 and reads locations[-1] for min-count <= 0.
    if (a.threads < 1) { fprintf(stderr, "[ERROR] -t must be >= 1\n"); exit(EXIT_FAILURE); }
    if (a.prm.consensus_min_count < 1) { fprintf(stderr, "[ERROR] --consensus-min-count must be >= 1\n"); exit(EXIT_FAILURE); }
    if (a.gpu_inflate < 0) {   // auto: small BAMs inflate faster on the host than the HIP start-up takes
        struct stat st;
        a.gpu_inflate = stat(a.bam, &st) == 0 && st.st_size >= (off_t)(1ll << 30) ? 1 : 0;
    }
    if (a.gpus < 1) a.gpus = 1;
    if (a.batch < 1) a.batch = 1;
    if (a.devices.empty())
        for (int g = 0; g < a.gpus; g++) a.devices.push_back(a.device + g);
    a.gpus = (int)a.devices.size();
    return a;
}

bool read_file(const char *path, std::string &s) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, k);
    fclose(f);
    return true;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One device's genomic shard: its loci (genomic order, VCF rows kept) and a copy of the
// reads their queries can yield.  Query hull per contig: A2 windows in uint32
// (audit.c:178,191-192), sam_itr_queryi(start-1, end-1) (refinement.c:114), empty when
// end <= beg; INV collects nothing (A7).  A read is kept when pos < hull.end and
// endpos > hull.beg -- a superset of every query's yield, so results are unchanged.
struct Shard {
    std::vector<size_t> rows;
    std::vector<svt_locus> loci;
    std::vector<svt_result> res;
    std::vector<int64_t> tid_off;
    std::vector<int32_t> pos, endpos;
    std::vector<uint64_t> cig_off;
    std::vector<uint32_t> cigar;
    std::vector<uint8_t> clip;
    svt_pileup_view view{};
};

void build_shard(const svt_pileup_view &full, const std::vector<svt_locus> &loci, const std::vector<size_t> &rows,
                 const svt_params &prm, Shard &sh) {
    sh.rows = rows;
    sh.loci.resize(rows.size());
    for (size_t k = 0; k < rows.size(); k++) sh.loci[k] = loci[rows[k]];
    sh.res.resize(rows.size());
    const int nt = full.n_targets;
    std::vector<int64_t> lo(nt, INT64_MAX), hi(nt, INT64_MIN);
    auto add = [&](const svt_locus &l, uint32_t s, uint32_t e) {
        int64_t b = (uint32_t)(s - 1u), q = (uint32_t)(e - 1u);
        int tid = l.chrom - 1;
        if (q <= b || tid < 0 || tid >= nt) return;
        lo[tid] = std::min(lo[tid], b);
        hi[tid] = std::max(hi[tid], q);
    };
    for (const svt_locus &l : sh.loci) {
        if (l.type == 1) add(l, l.pos - (uint32_t)prm.median_interval, l.pos + (uint32_t)prm.median_interval);
        if (l.type == 2) {
            add(l, l.pos - (uint32_t)prm.wider_interval, l.pos + (uint32_t)prm.narrow_interval);
            add(l, l.end - (uint32_t)prm.narrow_interval, l.end + (uint32_t)prm.narrow_interval);
        }
    }
    sh.tid_off.assign(1, 0);
    sh.cig_off.assign(1, 0);
    for (int t = 0; t < nt; t++) {
        int64_t a = full.tid_off[t], b = full.tid_off[t + 1];
        if (hi[t] > lo[t]) {
            const int32_t *cut = std::lower_bound(full.pos + a, full.pos + b, hi[t],
                                                  [](int32_t p, int64_t v) { return (int64_t)p < v; });
            for (int64_t r = a; r < cut - full.pos; r++) {
                if ((int64_t)full.endpos[r] <= lo[t]) continue;
                sh.pos.push_back(full.pos[r]);
                sh.endpos.push_back(full.endpos[r]);
                if (full.clip) sh.clip.push_back(full.clip[r]);
                sh.cigar.insert(sh.cigar.end(), full.cigar + full.cig_off[r], full.cigar + full.cig_off[r + 1]);
                sh.cig_off.push_back(sh.cigar.size());
            }
        }
        sh.tid_off.push_back((int64_t)sh.pos.size());
    }
    sh.view.n_targets = nt;
    sh.view.tid_off = sh.tid_off.data();
    sh.view.pos = sh.pos.data();
    sh.view.endpos = sh.endpos.data();
    sh.view.cig_off = sh.cig_off.data();
    sh.view.cigar = sh.cigar.data();
    sh.view.clip = full.clip ? sh.clip.data() : nullptr;
}

// The ingest's BGZF inflater on the first device (svt_bgzf_inflate), once its context is open.
struct DeviceInflate {
    std::shared_future<void> ready;
    svt_ctx **ctx;
    const int *open_rc;
    double ms = 0;   // device time of the inflate kernels
};
void *device_host_alloc(void *user, size_t bytes) {   // pinned buffers for the ingest's batches
    DeviceInflate *d = (DeviceInflate *)user;
    d->ready.wait();
    return *d->open_rc || !*d->ctx ? malloc(bytes) : svt_host_alloc(*d->ctx, bytes);
}
void device_host_free(void *user, void *p) {
    DeviceInflate *d = (DeviceInflate *)user;
    if (*d->open_rc || !*d->ctx) free(p);
    else svt_host_free(*d->ctx, p);
}
int device_inflate(void *user, const uint8_t *comp, size_t cb, const svt_bgzf_block *blocks, size_t n, uint8_t *out,
                   size_t ob, char *err, size_t ecap) {
    DeviceInflate *d = (DeviceInflate *)user;
    d->ready.wait();
    if (*d->open_rc || !*d->ctx) {
        snprintf(err, ecap, "BGZF inflate: svt_open failed (HIP device?)");
        return 1;
    }
    if (svt_bgzf_inflate(*d->ctx, comp, cb, blocks, n, out, ob) != SVT_OK) {
        snprintf(err, ecap, "BGZF inflate on the device: %s", svt_last_error(*d->ctx));
        return 1;
    }
    d->ms += svt_bgzf_last_inflate_ms(*d->ctx);
    return 0;
}

// The ingest's device sink (svt_bam_dec_*): BAM batches go to the first device compressed and
// are inflated and decoded there into the pileup (one device; --gpus N > 1 parses on the host).
struct DeviceDecode {
    std::shared_future<void> ready;
    svt_ctx **ctx;
    const int *open_rc;
    svt_bam_dec *dec = nullptr;
    // batch buffers in pageable host memory (SVTREK_DEC_PINNED=1: pinned).  Pinning two 256 MiB
    // buffers is on every run's critical path and costs more than the runtime's staged copies of
    // pageable memory: cfg4 contig 1.13-1.34 s pageable vs 1.54-1.60 s pinned (profiles/r04_batch2)
    bool pinned = false;
};
int dd_begin(void *user, int32_t n_targets, char *err, size_t ecap) {
    DeviceDecode *d = (DeviceDecode *)user;
    d->ready.wait();
    if (*d->open_rc || !*d->ctx) { snprintf(err, ecap, "BAM decode: svt_open failed (HIP device?)"); return 1; }
    if (svt_bam_dec_open(*d->ctx, n_targets, &d->dec) != SVT_OK) {
        snprintf(err, ecap, "BAM decode: %s", svt_last_error(*d->ctx));
        return 1;
    }
    return 0;
}
int dd_feed(void *user, const uint8_t *comp, size_t cb, const svt_bgzf_block *blocks, size_t n, uint64_t skip, char *err,
            size_t ecap) {
    DeviceDecode *d = (DeviceDecode *)user;
    if (svt_bam_dec_feed(d->dec, comp, cb, blocks, n, skip) != SVT_OK) {
        snprintf(err, ecap, "BAM decode on the device: %s", svt_last_error(*d->ctx));
        return 1;
    }
    return 0;
}
void *dd_alloc(void *user, size_t bytes) {
    DeviceDecode *d = (DeviceDecode *)user;
    d->ready.wait();
    return !d->pinned || *d->open_rc || !*d->ctx ? nullptr : svt_host_alloc(*d->ctx, bytes);   // nullptr: malloc
}
void dd_release(void *user, void *p) {
    DeviceDecode *d = (DeviceDecode *)user;
    svt_host_free(*d->ctx, p);
}

int audit(int argc, char **argv) {
    Args a = parse_audt(argc, argv);
    const double t0 = now_s();
    printf("[INFO] Started processing variation file.\n");
    fflush(stdout);

    // The GPU contexts (HIP runtime start-up, code object load) open beside the ingest too
    const int G = a.gpus;
    std::vector<svt_ctx *> ctxs(G, nullptr);
    std::vector<int> open_rc(G, 0);
    std::promise<void> first_open;
    DeviceInflate dinf{first_open.get_future().share(), &ctxs[0], &open_rc[0]};
    std::thread ot([&] {
        for (int g = 0; g < G; g++) {
            open_rc[g] = svt_open(&a.prm, a.devices[g], &ctxs[g]);
            if (g == 0) first_open.set_value();   // the ingest's inflater may start
        }
    });
    auto close_all = [&] {
        for (svt_ctx *c : ctxs)
            if (c) svt_close(c);
    };
    // BAM ingest and the VCF read + A1 parse are independent: the parse runs beside the ingest
    std::string vcf;
    bool vcf_ok = false;
    svth_vcf *pv = nullptr;
    double t_parse_end = 0;
    std::thread vt([&] {
        vcf_ok = read_file(a.vcf, vcf);
        if (vcf_ok) pv = svth_vcf_parse(vcf.data(), vcf.size(), a.threads);   // A1, audit.c:301-338
        t_parse_end = now_s();
    });
    char err[512];
    // GPU inflate: 1 GiB compressed batches (~21K BGZF blocks, one lane each; larger batches
    // inflate faster but pinning their buffers costs more: cfg2 e2e 5.4 s at 1 GiB, 9.0 s at 4 GiB)
    size_t batch_mb = 1024;
    // the device record decode: 256 MiB batches (pinned buffers: cfg4 contig 1 1.51 s at 256 MiB,
    // 1.79 at 512, 2.09 at 1 GiB, 1.54 / 1.82 at 128 / 64; cfg2 2.66 / 2.72 / 3.36 s; profiles/r04_batch*)
    size_t dec_batch_mb = 256;
    if (const char *x = getenv("SVTREK_INFLATE_BATCH_MB")) dec_batch_mb = batch_mb = std::max<size_t>(1, strtoull(x, nullptr, 10));
    const svth_inflater dev_inf{device_inflate, device_host_alloc, device_host_free, &dinf, batch_mb << 20};
    // one GPU: the records are decoded on the device too (svt_bam_dec_*; SVTREK_HOSTPARSE=1: the
    // device inflates, the host parses, as for --gpus N > 1)
    const char *hp = getenv("SVTREK_HOSTPARSE");
    const bool dev_decode = a.gpu_inflate && G == 1 && !(hp && atoi(hp) == 1);
    DeviceDecode ddec{dinf.ready, &ctxs[0], &open_rc[0]};
    if (const char *x = getenv("SVTREK_DEC_PINNED")) ddec.pinned = atoi(x) != 0;
    const svth_dev_sink dsink{dd_begin, dd_feed, dd_alloc, dd_release, &ddec, dec_batch_mb << 20};
    svth_bam *bam = nullptr;
    double dstage[4] = {0, 0, 0, 0};
    int dec_rc = 0;
    if (dev_decode) dec_rc = svth_bam_read_device(a.bam, a.threads, &dsink, nullptr, dstage, err, sizeof err);
    else bam = svth_bam_read_ex(a.bam, a.threads, -1, 0, -1, 0, a.gpu_inflate ? &dev_inf : nullptr, err, sizeof err);
    const double t_ingest = now_s();
    vt.join();
    ot.join();
    if (dev_decode ? dec_rc != 0 : !bam) {
        fprintf(stderr, "[ERROR] %s\n", err);
        svt_bam_dec_close(ddec.dec);
        svth_vcf_free(pv);
        close_all();
        return 1;
    }
    if (!vcf_ok) {
        fprintf(stderr, "[ERROR]: File couldn't be opened %s\n", a.vcf);
        svth_bam_free(bam);
        svt_bam_dec_close(ddec.dec);
        close_all();
        return 1;
    }
    double stage[6] = {0, 0, 0, 0, 0, 0};
    svt_pileup_view view{};
    if (bam) {
        svth_bam_stage_seconds(bam, stage);
        svth_bam_view(bam, &view);
    }
    size_t mlen = 0;
    const char *msgs = svth_vcf_messages(pv, &mlen);
    if (mlen) fwrite(msgs, 1, mlen, stderr);
    std::vector<svt_locus> loci(svth_vcf_loci(pv), svth_vcf_loci(pv) + svth_vcf_count(pv));
    svth_vcf_free(pv);
    std::string().swap(vcf);

    const double t_parse = now_s();
    std::vector<svt_result> res(loci.size());
    std::vector<int> rc(G, 0);
    std::vector<std::string> gerr(G);
    std::vector<double> load_s(G, 0.0);
    std::vector<size_t> order;
    svt_bam_dec_stats dst{};
    if (G > 1) {
        order.resize(loci.size());
        std::iota(order.begin(), order.end(), (size_t)0);
        std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
            return loci[x].chrom != loci[y].chrom ? loci[x].chrom < loci[y].chrom : loci[x].pos < loci[y].pos;
        });
    }
    auto worker = [&](int g) {
        svt_ctx *ctx = ctxs[g];
        int s = open_rc[g];
        if (s || !ctx) { rc[g] = s ? s : SVT_EDEVICE; gerr[g] = "svt_open failed (HIP device?)"; return; }
        const svt_locus *in = loci.data();
        svt_result *out = res.data();
        size_t n = loci.size();
        Shard sh;
        const double tl = now_s();
        if (G > 1) {
            size_t per = (n + G - 1) / G, b0 = std::min(n, per * (size_t)g), b1 = std::min(n, b0 + per);
            build_shard(view, loci, std::vector<size_t>(order.begin() + b0, order.begin() + b1), a.prm, sh);
            s = svt_load_pileup(ctx, &sh.view);
            in = sh.loci.data();
            out = sh.res.data();
            n = sh.loci.size();
        } else if (ddec.dec) {   // decoded on this device: its pileup, in place
            s = svt_bam_dec_load(ddec.dec);
            (void)svt_bam_dec_stats_get(ddec.dec, &dst);
            svt_bam_dec_close(ddec.dec);
            ddec.dec = nullptr;
        } else {
            s = svt_load_pileup(ctx, &view);
        }
        load_s[g] = now_s() - tl;
        for (size_t k = 0; !s && k < n; k += a.batch) {
            size_t m = std::min(a.batch, n - k);
            s = svt_refine_batch(ctx, in + k, m, out + k);
        }
        if (s) { rc[g] = s; gerr[g] = svt_last_error(ctx); }
        svt_close(ctx);
        ctxs[g] = nullptr;
        if (!s && G > 1)
            for (size_t k = 0; k < sh.rows.size(); k++) res[sh.rows[k]] = sh.res[k];
    };
    if (G == 1) worker(0);
    else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; g++) th.emplace_back(worker, g);
        for (auto &t : th) t.join();
    }
    for (int g = 0; g < G; g++)
        if (rc[g]) { fprintf(stderr, "[ERROR] GPU %d: %s (status %d)\n", a.devices[g], gerr[g].c_str(), rc[g]); return 1; }
    svth_bam_free(bam);
    const double t_refine = now_s();

    // A11, in VCF order
    size_t olen = 0;
    char *out = svth_format_batch(loci.data(), res.data(), loci.size(), a.threads, &olen);
    if (!out) { fprintf(stderr, "[ERROR] out of host memory\n"); return 1; }
    fwrite(out, 1, olen, stdout);
    svth_free(out);
    printf("[INFO] Ended processing variation file\n");
    if (a.verbose)   // --verbose is parsed but unused by the reference; here: stage timings on stderr
        fprintf(stderr, "[svtrek_amd] ingest %.3fs (%s%s)  vcf-read+parse %.3fs (beside the ingest)  "
                        "load+refine %.3fs (load %.3fs)  print %.3fs  records %zu%s\n",
                t_ingest - t0,
                dev_decode ? "gpu inflate + record decode" : a.gpu_inflate ? "gpu inflate, host parse, kernels " : "cpu",
                dev_decode ? ("; batch reads " + std::to_string(dstage[0]).substr(0, 5) + "s device feeds " +
                              std::to_string(dstage[1]).substr(0, 5) + "s waits " + std::to_string(dstage[2]).substr(0, 5) +
                              "s").c_str()
                : a.gpu_inflate ? (std::to_string(dinf.ms / 1e3).substr(0, 5) + "s; batch read " +
                                   std::to_string(stage[0]).substr(0, 5) + "s alloc " + std::to_string(stage[2]).substr(0, 5) +
                                   "s inflate calls " + std::to_string(stage[3]).substr(0, 5) + "s parser waits " +
                                   std::to_string(stage[4]).substr(0, 5) + "s").c_str() : "",
                t_parse_end - t0, t_refine - t_parse, *std::max_element(load_s.begin(), load_s.end()),
                now_s() - t_refine, loci.size(),
                dev_decode ? ("  decode: " + std::to_string(dst.batches) + " batches, " + std::to_string(dst.rechained) +
                              " re-chained (" + std::to_string(dst.rechained_chunks) + " chunks walked hop by hop)").c_str()
                           : "");
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        usage();
        exit(1);
    }
    if (strcmp(argv[1], "audt") == 0) {
        return audit(argc, argv);   // 0 on success; 1 on ingest/GPU errors (the reference crashes)
    }
    if (strcmp(argv[1], "disc") == 0) {
        fprintf(stderr, "[ERROR] disc mode is not part of svtrek_amd (it implements the audt path only)\n");
        return 1;
    }
    usage();
    exit(1);
}

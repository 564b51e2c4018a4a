// host_pipe.cpp -- pipelined host-memory batches.
//
// The reference's repair path starts and ends in host memory.  Helper
// sub-chunks arrive on sockets into ByteBuffers (ClayCoordinator.kt:372-395),
// and repaired sub-chunks leave the same way (ClayCodeNode.kt:330-347).
// run_host_batch takes the device batch layout with host pointers.  It streams
// chunks of stripes through a ring of device buffer sets on three streams, so
// the PCIe transfers of chunk i+1 and i-1 overlap the kernel of chunk i:
//
//   h2d stream:  [in i] [in i+1] ...      (waits: the kernel that last read set k)
//   cmp stream:         [map i]  ...      (waits: in i loaded, out i-NB drained)
//   d2h stream:                [out i] ...(waits: map i)
//
// Only the map's used input slots cross PCIe; the Clay(4,2) e=1 repair, for
// example, moves 20 of the 48 sub-chunks of a stripe.  Consecutive used slots
// that are also consecutive in host memory form a run; a chunk's copies are
// planned from the runs (make_plan): periodic runs folded into one 2D copy,
// other progressions of equal runs in one 3D copy each, a one-chunk batch of
// huge stripes cut into column slices, and over a device list, few stripes
// split by byte ranges (ecx_map_host_plan reports the plan).
#include <algorithm>
#include <cstring>
#include <thread>

#include "host_pipe.hpp"

namespace ecx {
namespace {

struct Run {
    int slot0;     // first host slot
    int compact0;  // first compact (device) slot
    int len;       // slots in the run
};

std::vector<Run> runs_of(const std::vector<int> &slots, int64_t slot_stride, int64_t nbytes) {
    std::vector<Run> runs;
    for (size_t i = 0; i < slots.size(); ++i) {
        if (!runs.empty() && slot_stride == nbytes && slots[i] == runs.back().slot0 + runs.back().len) {
            ++runs.back().len;
            continue;
        }
        runs.push_back({slots[i], (int)i, 1});
    }
    return runs;
}

// The runs of a stripe often repeat with a fixed step: a Clay repair reads the same helper nodes
// of every plane of a plane group (Clay(4,2) {0,3}: nodes 1-2 and 4-5 of all 8 planes, 16 runs;
// shortened Clay(10,4), node 0: nodes 1-13 of planes 0-63, 64 runs), a check on a padded pitch
// reads every shard.  One copy then moves many runs of every stripe of a chunk:
//  * folded 2D: when runs[i + period] is runs[i] moved by fixed host and compact steps for every i
//    and `count` steps span exactly one stripe on both sides, the k-th run of every period of
//    every stripe lies at a fixed pitch -- one strided copy of count x stripes rows per run of
//    the first period (Clay(4,2) {0,3}: 1 copy per chunk instead of 16, e2e 71.6 -> 75.9 GiB/s,
//    profiles/r06_fold_ab.jsonl);
//  * 3D: otherwise each maximal progression of equal runs at fixed steps (that divide the stripe
//    on both sides) is one hipMemcpy3DAsync -- its rows, then the next stripe (Clay(10,4) node 3:
//    3 copies per chunk instead of 65; H2D of node 0's 64 runs 53.2 -> 57.2 GB/s,
//    profiles/r06_copy3d_probe.jsonl; its e2e 56.7 -> 62.5 GiB/s, the headline's 68.0 -> 69.4,
//    profiles/r06_copy3d_ab.jsonl);
//  * any other run: one strided copy of its rows of the chunk's stripes.
struct Copy {
    int64_t host_off, dev_off;      // the copy's first byte in the chunk's first stripe
    int64_t width;                  // bytes per row
    int64_t rows;                   // rows per stripe
    int64_t host_pitch, dev_pitch;  // between a stripe's rows (folded: continuing across stripes)
    bool three_d;                   // rows of one stripe, then the next stripe a stripe stride on
};

std::vector<Copy> plan_copies(const std::vector<Run> &runs, int64_t stripe_stride, int64_t slot_stride, int64_t per,
                              int64_t nbytes) {
    std::vector<Copy> cs;
    const size_t n = runs.size();
    for (size_t p = 1; p < n; ++p) {  // folded 2D
        if (n % p) continue;
        const int64_t ds = runs[p].slot0 - runs[0].slot0, dc = runs[p].compact0 - runs[0].compact0;
        const int64_t count = (int64_t)(n / p);
        if (ds <= 0 || dc <= 0 || count * ds * slot_stride != stripe_stride || count * dc * nbytes != per) continue;
        bool ok = true;
        for (size_t i = 0; ok && i + p < n; ++i)
            ok = runs[i + p].len == runs[i].len && runs[i + p].slot0 - runs[i].slot0 == ds &&
                 runs[i + p].compact0 - runs[i].compact0 == dc;
        if (!ok) continue;
        for (size_t k = 0; k < p; ++k)
            cs.push_back({runs[k].slot0 * slot_stride, runs[k].compact0 * nbytes, runs[k].len * nbytes, count,
                          ds * slot_stride, dc * nbytes, false});
        return cs;
    }
    for (size_t i = 0; i < n;) {
        size_t j = i;
        int64_t ds = 0, dc = 0;
        if (i + 1 < n && runs[i + 1].len == runs[i].len) {
            ds = runs[i + 1].slot0 - runs[i].slot0;
            dc = runs[i + 1].compact0 - runs[i].compact0;
            while (j + 1 < n && runs[j + 1].len == runs[i].len && runs[j + 1].slot0 - runs[j].slot0 == ds &&
                   runs[j + 1].compact0 - runs[j].compact0 == dc)
                ++j;
        }
        const int64_t hp = ds * slot_stride, dp = dc * nbytes;
        if (j > i && hp > 0 && dp > 0 && stripe_stride > 0 && stripe_stride % hp == 0 &&
            per % dp == 0) {
            cs.push_back({runs[i].slot0 * slot_stride, runs[i].compact0 * nbytes, runs[i].len * nbytes,
                          (int64_t)(j - i + 1), hp, dp, true});
        } else {
            for (size_t k = i; k <= j; ++k)
                cs.push_back({runs[k].slot0 * slot_stride, runs[k].compact0 * nbytes, runs[k].len * nbytes, 1,
                              stripe_stride, per, false});
        }
        i = j + 1;
    }
    return cs;
}

// A progression of equal runs -- runs i..j of one length, `ds` host slots and `dc` compact slots
// apart -- for the column-sliced copies below.
struct Segment {
    size_t i, j;
    int64_t ds, dc;
};

std::vector<Segment> segments_of(const std::vector<Run> &runs) {
    std::vector<Segment> sg;
    for (size_t i = 0; i < runs.size();) {
        size_t j = i;
        int64_t ds = 0, dc = 0;
        if (i + 1 < runs.size() && runs[i + 1].len == runs[i].len) {
            ds = runs[i + 1].slot0 - runs[i].slot0;
            dc = runs[i + 1].compact0 - runs[i].compact0;
            while (j + 1 < runs.size() && runs[j + 1].len == runs[i].len && runs[j + 1].slot0 - runs[j].slot0 == ds &&
                   runs[j + 1].compact0 - runs[j].compact0 == dc)
                ++j;
        }
        sg.push_back({i, j, ds, dc});
        i = j + 1;
    }
    return sg;
}

// The chunking and copy plan of one host batch (run_host_batch; run_host_check_batch, whose only
// output is one verdict byte per stripe).  A batch whose stripes all fit one chunk but carry far
// more than a chunk of input (config 4 with 1 MiB sub-chunks: one 3.5 GiB stripe per call) is cut
// into column slices instead -- bytes [c0, c0 + slice) of every slot, the map being bytewise --
// so its H2D, kernel and D2H still overlap, the way the reference's repair pipelining slices a
// block (PipelineUtil.kt:13-28).
struct Plan {
    std::vector<Run> rin, rout;
    std::vector<Copy> cin, cout;
    std::vector<Segment> sin, sout;  // the runs' progressions, for column slices
    int64_t in_per = 0, out_per = 0, chunk = 1, nchunks = 0;
    int64_t slice = 0, nslices = 1;  // column slices (slice 0: whole slots)
    int nb = 1;
};

Plan make_plan(CompiledMap &cm, int64_t in_stripe_stride, int64_t in_slot_stride, int64_t out_stripe_stride,
               int64_t out_slot_stride, int64_t nstripes, int64_t nbytes, bool outputs) {
    Plan pl;
    const std::vector<int> &ins = cm.used_in_slots();
    pl.in_per = (int64_t)ins.size() * nbytes;
    pl.rin = runs_of(ins, in_slot_stride, nbytes);
    if (outputs) {
        const std::vector<int> &outs = cm.used_out_slots();
        pl.out_per = (int64_t)outs.size() * nbytes;
        pl.rout = runs_of(outs, out_slot_stride, nbytes);
    }
    const Tuning &t = tuning();
    const int64_t in_per = pl.in_per;
    const std::vector<Run> &rin = pl.rin;
    // Stripes per chunk: host_chunk bytes of input, but at least kMinRows stripes when a chunk still
    // takes more than 8 copies after folding and 3D (Clay(10,4) node 4: 17), so each copy moves rows
    // of many stripes instead of a few KiB -- within 8x host_chunk.  The DMA queue idles ~16 us
    // between copies (the copy trace); with one copy per run, 160 rows beat 64, 96, 256
    // and 512 and equal-size chunks (profiles/r06_minrows_ab*.jsonl); once 3D copies took Clay(10,4)
    // node 3 to 3 copies, dropping the floor for it gained another 4 % (profiles/r06_floor_ab.jsonl).
    constexpr int64_t kMinRows = 160;
    pl.cin = plan_copies(rin, in_stripe_stride, in_slot_stride, in_per, nbytes);
    int64_t chunk = t.host_chunk / std::max<int64_t>(1, in_per);
    if (pl.cin.size() > 8) chunk = std::max(chunk, std::min(kMinRows, 8 * t.host_chunk / std::max<int64_t>(1, in_per)));
    chunk = std::max<int64_t>(1, std::min<int64_t>(nstripes, chunk));
    const int64_t nchunks = (nstripes + chunk - 1) / chunk;
    pl.chunk = chunk;
    pl.nchunks = nchunks;
    pl.nb = (int)std::min<int64_t>(std::max(1, std::min(t.host_buffers, 8)), std::max<int64_t>(1, nchunks));
    if (outputs) pl.cout = plan_copies(pl.rout, out_stripe_stride, out_slot_stride, pl.out_per, nbytes);
    constexpr int64_t kSliceAlign = 4096;
    if (outputs && nchunks == 1 && nbytes >= 2 * kSliceAlign && nstripes * in_per >= 4 * t.host_chunk) {
        const int64_t want = (nstripes * in_per + t.host_chunk - 1) / t.host_chunk;  // slices of ~host_chunk
        int64_t w = (nbytes + want - 1) / want;
        w = (w + kSliceAlign - 1) / kSliceAlign * kSliceAlign;
        pl.slice = std::min(w, nbytes);
        pl.nslices = (nbytes + pl.slice - 1) / pl.slice;
        pl.sin = segments_of(rin);
        pl.sout = segments_of(pl.rout);
        pl.nb = (int)std::min<int64_t>(std::max(1, std::min(t.host_buffers, 8)), pl.nslices);
    }
    return pl;
}

// Copy `rows` rows of `width` bytes between two pitched layouts.
void copy_rows(uint8_t *dst, int64_t dpitch, const uint8_t *src, int64_t spitch, int64_t width, int64_t rows,
               hipMemcpyKind kind, hipStream_t s) {
    if (rows == 1 || (dpitch == width && spitch == width)) {
        check_hip(hipMemcpyAsync(dst, src, (size_t)(width * rows), kind, s), "hipMemcpyAsync (host batch)");
        return;
    }
    if (dpitch >= width && spitch >= width) {
        check_hip(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)rows, kind, s),
                  "hipMemcpy2DAsync (host batch)");
        return;
    }
    for (int64_t r = 0; r < rows; ++r)
        check_hip(hipMemcpyAsync(dst + r * dpitch, src + r * spitch, (size_t)width, kind, s),
                  "hipMemcpyAsync (host batch row)");
}

// One planned copy for the `n` stripes of a chunk: host side at `host` (stripe stride
// `host_stripe`), device side at `dev` (stripe stride `dev_stripe`), in direction `kind`.
void issue_copy(const Copy &c, const uint8_t *host_base, uint8_t *dev_base, int64_t host_stripe, int64_t dev_stripe,
                int64_t n, hipMemcpyKind kind, hipStream_t s) {
    uint8_t *host = const_cast<uint8_t *>(host_base) + c.host_off;
    uint8_t *dev = dev_base + c.dev_off;
    const bool h2d = kind == hipMemcpyHostToDevice;
    if (c.three_d) {
        hipMemcpy3DParms p;
        std::memset(&p, 0, sizeof(p));
        const hipPitchedPtr hptr = make_hipPitchedPtr(host, (size_t)c.host_pitch, (size_t)c.width,
                                                      (size_t)(host_stripe / c.host_pitch));
        const hipPitchedPtr dptr = make_hipPitchedPtr(dev, (size_t)c.dev_pitch, (size_t)c.width,
                                                      (size_t)(dev_stripe / c.dev_pitch));
        p.srcPtr = h2d ? hptr : dptr;
        p.dstPtr = h2d ? dptr : hptr;
        p.extent = make_hipExtent((size_t)c.width, (size_t)c.rows, (size_t)n);
        p.kind = kind;
        if (hipMemcpy3DAsync(&p, s) == hipSuccess) return;
        (void)hipGetLastError();  // refused shape (nothing enqueued): the same rows as per-stripe 2D copies
        for (int64_t t = 0; t < n; ++t)
            copy_rows(h2d ? dev + t * dev_stripe : host + t * host_stripe, h2d ? c.dev_pitch : c.host_pitch,
                      h2d ? host + t * host_stripe : dev + t * dev_stripe, h2d ? c.host_pitch : c.dev_pitch, c.width,
                      c.rows, kind, s);
        return;
    }
    if (h2d) copy_rows(dev, c.dev_pitch, host, c.host_pitch, c.width, n * c.rows, kind, s);
    else copy_rows(host, c.host_pitch, dev, c.dev_pitch, c.width, n * c.rows, kind, s);
}

// Bytes [c0, c0 + w) of every used slot of `n` stripes between the host layout (stripe stride
// host_stripe, slot stride slot_stride) and a compact device slice ([stripe][used slot][w]): per
// stripe, each progression of runs is one 3D copy -- w bytes of each of a run's slots (slot_stride
// apart), runs ds slots apart -- or a 2D copy for a lone run.
void issue_sliced(const std::vector<Run> &runs, const std::vector<Segment> &segs, const uint8_t *host_base,
                  uint8_t *dev_base, int64_t host_stripe, int64_t slot_stride, int64_t used, int64_t n, int64_t w,
                  hipMemcpyKind kind, hipStream_t s) {
    const bool h2d = kind == hipMemcpyHostToDevice;
    for (int64_t t = 0; t < n; ++t)
        for (const Segment &g : segs) {
            const Run &r = runs[g.i];
            uint8_t *host = const_cast<uint8_t *>(host_base) + t * host_stripe + r.slot0 * slot_stride;
            uint8_t *dev = dev_base + (t * used + r.compact0) * w;
            if (g.j > g.i) {
                hipMemcpy3DParms p;
                std::memset(&p, 0, sizeof(p));
                const hipPitchedPtr hptr = make_hipPitchedPtr(host, (size_t)slot_stride, (size_t)w, (size_t)g.ds);
                const hipPitchedPtr dptr = make_hipPitchedPtr(dev, (size_t)w, (size_t)w, (size_t)g.dc);
                p.srcPtr = h2d ? hptr : dptr;
                p.dstPtr = h2d ? dptr : hptr;
                p.extent = make_hipExtent((size_t)w, (size_t)r.len, g.j - g.i + 1);
                p.kind = kind;
                if (hipMemcpy3DAsync(&p, s) == hipSuccess) continue;
                (void)hipGetLastError();  // refused shape (nothing enqueued): run by run
            }
            for (size_t k = g.i; k <= g.j; ++k) {
                uint8_t *hk = host + (runs[k].slot0 - r.slot0) * slot_stride;
                uint8_t *dk = dev + (runs[k].compact0 - r.compact0) * w;
                if (h2d) copy_rows(dk, w, hk, slot_stride, w, runs[k].len, kind, s);
                else copy_rows(hk, slot_stride, dk, w, w, runs[k].len, kind, s);
            }
        }
}

// Per-device streams, buffer sets and events of the host-batch pipeline.
class HostPipe {
public:
    struct Set {
        uint8_t *in = nullptr, *out = nullptr;
        size_t in_cap = 0, out_cap = 0;
        hipEvent_t loaded = nullptr, computed = nullptr, drained = nullptr;
    };

    static HostPipe &current() {
        static std::mutex reg_mu;
        static std::map<int, std::unique_ptr<HostPipe>> reg;
        int dev = 0;
        check_hip(hipGetDevice(&dev), "hipGetDevice");
        std::lock_guard<std::mutex> lk(reg_mu);
        auto &slot = reg[dev];
        if (!slot) {
            auto p = std::make_unique<HostPipe>();
            for (hipStream_t *s : {&p->h2d, &p->cmp, &p->d2h})
                check_hip(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate (host batch)");
            slot = std::move(p);
        }
        return *slot;
    }

    // Called with every stream idle (the previous call synchronised).
    void ensure(int nb, size_t in_bytes, size_t out_bytes) {
        while ((int)sets.size() < nb) {
            Set s;
            for (hipEvent_t *e : {&s.loaded, &s.computed, &s.drained})
                check_hip(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate (host batch)");
            sets.push_back(s);
        }
        for (int k = 0; k < nb; ++k) {
            Set &s = sets[k];
            if (s.in_cap < in_bytes) {
                if (s.in) check_hip(hipFree(s.in), "hipFree (host batch)");
                s.in = nullptr;
                s.in_cap = 0;
                check_hip(hipMalloc(&s.in, in_bytes), "hipMalloc (host batch)");
                s.in_cap = in_bytes;
            }
            if (s.out_cap < out_bytes) {
                if (s.out) check_hip(hipFree(s.out), "hipFree (host batch)");
                s.out = nullptr;
                s.out_cap = 0;
                check_hip(hipMalloc(&s.out, out_bytes), "hipMalloc (host batch)");
                s.out_cap = out_bytes;
            }
        }
    }

    void drain() {
        for (hipStream_t s : {h2d, cmp, d2h}) (void)hipStreamSynchronize(s);
    }

    std::mutex mu;
    hipStream_t h2d = nullptr, cmp = nullptr, d2h = nullptr;
    std::vector<Set> sets;
};

}  // namespace

void run_host_batch(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                    uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                    int64_t nbytes) {
    if (nstripes <= 0 || nbytes <= 0 || cm.map().n_out == 0) return;
    CompiledMap &cc = cm.compact();
    const Plan pl = make_plan(cm, in_stripe_stride, in_slot_stride, out_stripe_stride, out_slot_stride, nstripes,
                              nbytes, true);
    const int64_t in_per = pl.in_per, out_per = pl.out_per, chunk = pl.chunk;
    const int nb = pl.nb;
    const bool sliced = pl.nslices > 1;
    const int64_t units = sliced ? pl.nslices : pl.nchunks;
    const int64_t used_in = (int64_t)cm.used_in_slots().size(), used_out = (int64_t)cm.used_out_slots().size();

    HostPipe &p = HostPipe::current();
    std::lock_guard<std::mutex> lk(p.mu);
    try {
        if (sliced) p.ensure(nb, (size_t)(nstripes * used_in * pl.slice), (size_t)(nstripes * used_out * pl.slice));
        else p.ensure(nb, (size_t)(chunk * in_per), (size_t)(chunk * out_per));
        for (int64_t i = 0; i < units; ++i) {
            HostPipe::Set &b = p.sets[(size_t)(i % nb)];
            // a chunk of whole-slot stripes, or (sliced) bytes [c0, c0 + w) of every stripe
            const int64_t lo = sliced ? 0 : i * chunk, n = sliced ? nstripes : std::min(chunk, nstripes - lo);
            const int64_t c0 = sliced ? i * pl.slice : 0, w = sliced ? std::min(pl.slice, nbytes - c0) : nbytes;
            const int64_t in_ss = sliced ? used_in * w : in_per, out_ss = sliced ? used_out * w : out_per;
            if (i >= nb) check_hip(hipStreamWaitEvent(p.h2d, b.computed, 0), "hipStreamWaitEvent");
            if (sliced)
                issue_sliced(pl.rin, pl.sin, in + c0, b.in, in_stripe_stride, in_slot_stride, used_in, n, w,
                             hipMemcpyHostToDevice, p.h2d);
            else
                for (const Copy &c : pl.cin)
                    issue_copy(c, in + lo * in_stripe_stride, b.in, in_stripe_stride, in_per, n, hipMemcpyHostToDevice,
                               p.h2d);
            check_hip(hipEventRecord(b.loaded, p.h2d), "hipEventRecord");
            check_hip(hipStreamWaitEvent(p.cmp, b.loaded, 0), "hipStreamWaitEvent");
            if (i >= nb) check_hip(hipStreamWaitEvent(p.cmp, b.drained, 0), "hipStreamWaitEvent");
            launch_apply(cc, b.in, in_ss, w, b.out, out_ss, w, n, w, p.cmp);
            check_hip(hipEventRecord(b.computed, p.cmp), "hipEventRecord");
            check_hip(hipStreamWaitEvent(p.d2h, b.computed, 0), "hipStreamWaitEvent");
            if (sliced)
                issue_sliced(pl.rout, pl.sout, out + c0, b.out, out_stripe_stride, out_slot_stride, used_out, n, w,
                             hipMemcpyDeviceToHost, p.d2h);
            else
                for (const Copy &c : pl.cout)
                    issue_copy(c, out + lo * out_stripe_stride, b.out, out_stripe_stride, out_per, n,
                               hipMemcpyDeviceToHost, p.d2h);
            check_hip(hipEventRecord(b.drained, p.d2h), "hipEventRecord");
        }
        check_hip(hipStreamSynchronize(p.d2h), "hipStreamSynchronize (host batch)");
    } catch (...) {
        p.drain();
        throw;
    }
}

HostBatchPlan plan_host_batch(CompiledMap &cm, int64_t in_stripe_stride, int64_t in_slot_stride,
                              int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes, int64_t nbytes) {
    HostBatchPlan hp;
    if (nstripes <= 0 || nbytes <= 0 || cm.map().n_out == 0) return hp;  // run_host_batch moves nothing
    const Plan pl = make_plan(cm, in_stripe_stride, in_slot_stride, out_stripe_stride, out_slot_stride, nstripes,
                              nbytes, true);
    hp.chunk = pl.chunk;
    hp.nchunks = pl.nchunks;
    hp.buffers = pl.nb;
    hp.h2d_copies = (int64_t)pl.cin.size();
    hp.d2h_copies = (int64_t)pl.cout.size();
    for (const Copy &c : pl.cin) hp.h2d_rows = std::max(hp.h2d_rows, c.rows), hp.h2d_3d += c.three_d;
    for (const Copy &c : pl.cout) hp.d2h_rows = std::max(hp.d2h_rows, c.rows), hp.d2h_3d += c.three_d;
    hp.slices = pl.nslices;
    if (pl.nslices > 1) {  // per slice: a copy per progression per stripe
        hp.buffers = pl.nb;
        hp.h2d_copies = (int64_t)pl.sin.size() * nstripes;
        hp.d2h_copies = (int64_t)pl.sout.size() * nstripes;
    }
    return hp;
}

void run_host_check_batch(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                          int64_t nstripes, int64_t nbytes, uint8_t *verdict) {
    if (nstripes <= 0) return;
    if (!verdict) throw Error(ECX_E_NULL, "verdict buffer is null");
    if (nbytes <= 0 || cm.map().n_out == 0) {  // nothing to compare: every stripe passes (as launch_check)
        std::memset(verdict, 1, (size_t)nstripes);
        return;
    }
    // The read-only twin of run_host_batch: the check map's used slots cross PCIe into a set's
    // compact buffer, k_gf_check writes one verdict byte per stripe of the chunk into the set's
    // output area, and only those bytes come back.
    CompiledMap &cc = cm.compact();
    const Plan pl = make_plan(cm, in_stripe_stride, in_slot_stride, 0, 0, nstripes, nbytes, false);
    const int64_t in_per = pl.in_per, chunk = pl.chunk, nchunks = pl.nchunks;
    const int nb = pl.nb;

    HostPipe &p = HostPipe::current();
    std::lock_guard<std::mutex> lk(p.mu);
    try {
        p.ensure(nb, (size_t)(chunk * in_per), (size_t)chunk);
        for (int64_t i = 0; i < nchunks; ++i) {
            HostPipe::Set &b = p.sets[(size_t)(i % nb)];
            const int64_t lo = i * chunk, n = std::min(chunk, nstripes - lo);
            if (i >= nb) check_hip(hipStreamWaitEvent(p.h2d, b.computed, 0), "hipStreamWaitEvent");
            for (const Copy &c : pl.cin)
                issue_copy(c, in + lo * in_stripe_stride, b.in, in_stripe_stride, in_per, n, hipMemcpyHostToDevice, p.h2d);
            check_hip(hipEventRecord(b.loaded, p.h2d), "hipEventRecord");
            check_hip(hipStreamWaitEvent(p.cmp, b.loaded, 0), "hipStreamWaitEvent");
            if (i >= nb) check_hip(hipStreamWaitEvent(p.cmp, b.drained, 0), "hipStreamWaitEvent");
            launch_check(cc, b.in, in_per, nbytes, b.out, n, nbytes, p.cmp);
            check_hip(hipEventRecord(b.computed, p.cmp), "hipEventRecord");
            check_hip(hipStreamWaitEvent(p.d2h, b.computed, 0), "hipStreamWaitEvent");
            check_hip(hipMemcpyAsync(verdict + lo, b.out, (size_t)n, hipMemcpyDeviceToHost, p.d2h),
                      "hipMemcpyAsync (verdicts)");
            check_hip(hipEventRecord(b.drained, p.d2h), "hipEventRecord");
        }
        check_hip(hipStreamSynchronize(p.d2h), "hipStreamSynchronize (host check batch)");
    } catch (...) {
        p.drain();
        throw;
    }
}

void stripe_range(int64_t nstripes, int parts, int j, int64_t *begin, int64_t *end) {
    // contiguous ranges, the remainder on the first ones (shard_stripes, __init__.py)
    const int64_t base = nstripes / parts, extra = nstripes % parts;
    *begin = j * base + std::min<int64_t>(j, extra);
    *end = *begin + base + (j < extra ? 1 : 0);
}

namespace {

// One worker thread per device entry over contiguous stripe ranges; `range(lo, n)` runs on the
// worker with its device current.  Bad ids are refused before any worker starts; the first
// failing device's status is thrown after every worker has joined (each drains its own pipe).
template <typename F>
void on_devices(const int *devices, int ndev, int64_t nstripes, F &&range) {
    if (!devices) throw Error(ECX_E_NULL, "null device list");
    if (ndev <= 0) throw Error(ECX_E_ILLEGAL_ARGUMENT, "empty device list");
    int count = 0;
    check_hip(hipGetDeviceCount(&count), "hipGetDeviceCount");
    for (int j = 0; j < ndev; ++j)
        if (devices[j] < 0 || devices[j] >= count)
            throw Error(ECX_E_ILLEGAL_ARGUMENT, "device " + std::to_string(devices[j]) + " of " +
                                                    std::to_string(count) + " visible");
    if (nstripes <= 0) return;
    struct Result {
        int code = ECX_OK;
        std::string what;
    };
    std::vector<Result> res((size_t)ndev);
    auto work = [&](int j) {
        int64_t lo = 0, hi = 0;
        stripe_range(nstripes, ndev, j, &lo, &hi);
        if (hi <= lo) return;
        try {
            check_hip(hipSetDevice(devices[j]), "hipSetDevice (host batch worker)");
            range(lo, hi - lo);
        } catch (const Error &e) {
            res[(size_t)j] = {e.code, e.what()};
        } catch (const std::bad_alloc &) {
            res[(size_t)j] = {ECX_E_NOMEM, "out of memory"};
        } catch (const std::exception &e) {
            res[(size_t)j] = {ECX_E_ILLEGAL_ARGUMENT, e.what()};
        }
    };
    // the caller's thread (and its current device) only waits
    std::vector<std::thread> th;
    th.reserve((size_t)ndev);
    try {
        for (int j = 0; j < ndev; ++j) th.emplace_back(work, j);
    } catch (...) {
        for (std::thread &t : th) t.join();
        throw Error(ECX_E_NOMEM, "cannot start a host-batch worker thread");
    }
    for (std::thread &t : th) t.join();
    for (int j = 0; j < ndev; ++j)
        if (res[(size_t)j].code != ECX_OK)
            throw Error(res[(size_t)j].code, "device " + std::to_string(devices[j]) + ": " + res[(size_t)j].what);
}

}  // namespace

void for_device_ranges(const int *devices, int ndev, int64_t nstripes,
                       const std::function<void(int64_t, int64_t)> &range) {
    on_devices(devices, ndev, nstripes, range);
}

void run_host_batch_devices(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride, int64_t in_slot_stride,
                            uint8_t *out, int64_t out_stripe_stride, int64_t out_slot_stride, int64_t nstripes,
                            int64_t nbytes, const int *devices, int ndev) {
    if (nbytes <= 0 || cm.map().n_out == 0) nstripes = 0;  // validate the list, touch nothing
    // Fewer stripes than device entries (one or two huge stripes): split the bytes of every slot
    // instead, in 4 KiB units -- the map is bytewise -- so every entry's link still carries a share.
    constexpr int64_t kColUnit = 4096;
    if (nstripes > 0 && nstripes < ndev && nbytes >= 2 * kColUnit) {
        on_devices(devices, ndev, (nbytes + kColUnit - 1) / kColUnit, [&](int64_t u0, int64_t nu) {
            const int64_t c0 = u0 * kColUnit, w = std::min(nu * kColUnit, nbytes - c0);
            run_host_batch(cm, in + c0, in_stripe_stride, in_slot_stride, out + c0, out_stripe_stride, out_slot_stride,
                           nstripes, w);
        });
        return;
    }
    on_devices(devices, ndev, nstripes, [&](int64_t lo, int64_t n) {
        run_host_batch(cm, in + lo * in_stripe_stride, in_stripe_stride, in_slot_stride, out + lo * out_stripe_stride,
                       out_stripe_stride, out_slot_stride, n, nbytes);
    });
}

void run_host_check_batch_devices(CompiledMap &cm, const uint8_t *in, int64_t in_stripe_stride,
                                  int64_t in_slot_stride, int64_t nstripes, int64_t nbytes, uint8_t *verdict,
                                  const int *devices, int ndev) {
    if (nstripes > 0 && !verdict) throw Error(ECX_E_NULL, "verdict buffer is null");
    // Fewer stripes than entries: each entry checks a byte range of every slot into its own
    // verdicts, and a stripe passes when it passes in every range.
    constexpr int64_t kColUnit = 4096;
    if (nstripes > 0 && nstripes < ndev && nbytes >= 2 * kColUnit && cm.map().n_out > 0) {
        const int64_t units = (nbytes + kColUnit - 1) / kColUnit;
        std::vector<std::vector<uint8_t>> part((size_t)ndev);
        on_devices(devices, ndev, units, [&](int64_t u0, int64_t nu) {
            int j = 0;  // this range's entry: the one whose range starts at u0
            for (int64_t b = 0, e = 0; j < ndev; ++j) {
                stripe_range(units, ndev, j, &b, &e);
                if (b == u0 && e > b) break;
            }
            std::vector<uint8_t> &v = part[(size_t)j];
            v.assign((size_t)nstripes, 0);
            const int64_t c0 = u0 * kColUnit, w = std::min(nu * kColUnit, nbytes - c0);
            run_host_check_batch(cm, in + c0, in_stripe_stride, in_slot_stride, nstripes, w, v.data());
        });
        std::memset(verdict, 1, (size_t)nstripes);
        for (const std::vector<uint8_t> &v : part)
            for (size_t s2 = 0; s2 < v.size(); ++s2) verdict[s2] = (uint8_t)(verdict[s2] && v[s2]);
        return;
    }
    on_devices(devices, ndev, nstripes, [&](int64_t lo, int64_t n) {
        run_host_check_batch(cm, in + lo * in_stripe_stride, in_stripe_stride, in_slot_stride, n, nbytes,
                             verdict + lo);
    });
}

}  // namespace ecx

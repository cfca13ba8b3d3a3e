// lower_bench.cpp -- what the Go shim pays per Eval before the device sees a
// job: the product's C++ lowering (include/reflow_host.hpp, reflow_host.cpp)
// of a 1000align-shaped Flow graph built with the reference's node shapes
// (doc/1000align: per pair Val -> Coerce -> Exec(bwa) -> Coerce -> K -> ... ;
// per sample K(P) -> Coerce -> Exec(merge) -> Coerce -> Extern), timed phase
// by phase:
//   build         the Flow nodes (a program's evaluation would create them)
//   canonicalize  reflow::Canonicalize (flow.go:814-843): copies, their digests
//                 on the device (an Eval over the copies: lowered on host
//                 threads, loaded, recomputed), flowMap dedup (K5)
//   lower         Eval::Add: materials + holes for every logical and physical
//                 job (flow.go:675-792) -- 0 when Canonicalize handed its Eval
//                 over (nothing collapsed: it is the canonical graph's)
//   load          Eval::Build: blob assembly, rf_graph_load, the File-ID
//                 inputs, one full recompute (0 likewise)
//   incremental   1% of the File IDs replaced (Eval::SetFileID) + Recompute,
//                 checked slot for slot against a full recompute
// With "dup" (a third argument) every sample builds its own copy of the
// reference-index chain (Intern -> Exec(bwa index) -> Coerce): equal digests,
// so Canonicalize collapses 3 x (samples - 1) copies and hands over its Eval
// with the duplicates' jobs dropped ("collapsed"); the canonical root digest
// equals the shared-chain graph's.
// Output: one JSON object on stdout.  usage: lower_bench <samples> <pairs> [dup]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "reflow_host.hpp"

using namespace reflow;
using Clock = std::chrono::steady_clock;

static double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

static Digest id_of(uint64_t tag, uint64_t i) {  // synthetic File IDs (splitmix64 stream)
    Digest d;
    uint64_t x = tag * 0x9E3779B97F4A7C15ull + i * 4;
    for (int k = 0; k < 4; ++k) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(d.b.data() + 8 * k, &z, 8);
    }
    return d;
}

static Digest fd(const char* s) {  // a FlowDigest constant (K / Coerce)
    Digest d = id_of(0xFD, (uint64_t)std::hash<std::string>{}(s));
    return d;
}

static int lower_threads_in_use(Engine& e) {
    if (const char* v = getenv("RF_LOWER_THREADS")) return atoi(v);
    int th = 0, ext = 0;
    double rate = 0;
    return rf_host_info(e.ctx(), &th, &rate, &ext) == RF_OK ? th : 0;
}

static Fileset one(const Digest& id) {
    Fileset v;
    v.Map["."] = File{id, 1};
    return v;
}

// Canonicalize's post-order and copy loop (reflow_host.cpp) on host threads,
// timed: whole copies, and copies without their Fileset values.
static int copy_probe(Flow* top, unsigned th) {
    auto t0 = Clock::now();
    std::vector<Flow*> post;
    detail::PtrIndex index;
    detail::PostOrder(top, th, post, index);
    const double t_walk = secs(t0);
    const size_t n = post.size();
    for (int variant = 0; variant < 2; ++variant) {
        FlowArena arena;
        t0 = Clock::now();
        arena.NewN(n, [&](Flow* blk, size_t, size_t) {
            std::vector<std::thread> pool;
            for (unsigned t = 0; t < th; ++t)
                pool.emplace_back([&, t] {
                    for (size_t i = n * t / th; i < n * (t + 1) / th; ++i) {
                        Flow* c = variant ? new (blk + i) Flow() : new (blk + i) Flow(*post[i]);
                        if (variant) {  // the fields without the value
                            const Flow& o = *post[i];
                            c->op = o.op;
                            c->Parent = o.Parent;
                            c->Deps = o.Deps;
                            c->Image = o.Image;
                            c->Cmd = o.Cmd;
                            c->URL = o.URL;
                            c->Argmap = o.Argmap;
                            c->FlowDigest = o.FlowDigest;
                            c->Done = o.Done;
                        }
                        for (Flow*& d : c->Deps) d = blk + *index.find(d);
                    }
                });
            for (auto& x : pool) x.join();
        });
        printf("{\"nodes\": %zu, \"threads\": %u, \"walk_s\": %.3f, \"copy_s\": %.3f, \"values\": %s}\n", n, th,
               t_walk, secs(t0), variant ? "false" : "true");
    }
    return 0;
}

int main(int argc, char** argv) {
    const uint64_t S = argc > 1 ? strtoull(argv[1], nullptr, 10) : 22075, P = argc > 2 ? strtoull(argv[2], nullptr, 10) : 32;
    const bool dup = argc > 3 && std::string(argv[3]) == "dup";
    // "copyprobe" (a diagnostic, host only -- no device): the graph built,
    // then Canonicalize's walk and copy loop timed on host threads, whole
    // nodes and without their Fileset values
    const bool copyprobe = argc > 3 && std::string(argv[3]) == "copyprobe";
    std::unique_ptr<Engine> eng;
    if (!copyprobe) eng = std::make_unique<Engine>(0);
    FlowArena a;
    auto t0 = Clock::now();
    const Digest fd_coerce = fd("file.fs$file"), fd_force = fd("Eval.Force"), fd_fs = fd("coerceFlowToFileset"),
                 fd_out = fd("coerceExecOutput"), fd_merge = fd("Force.merge");
    auto op1 = [&](Op op, Flow* dep, const Digest& d, const FlowValue& v) {
        Flow f;
        f.op = op;
        f.Deps = {dep};
        f.FlowDigest = d;
        f.Done = true;
        f.Value = v;
        return a.New(std::move(f));
    };
    auto exec = [&](const std::string& image, const std::string& cmd, std::vector<Flow*> deps, const Digest& out) {
        Flow* x = flow::Exec(a, image, cmd, std::move(deps));
        x->Argmap = std::vector<ExecArg>{};
        for (size_t i = 0; i < x->Deps.size(); ++i) x->Argmap->push_back(ExecArg{false, (int)i});
        x->Argmap->push_back(ExecArg{true, 0});
        x->Done = true;
        x->Value = one(out);
        return x;
    };
    auto ref_chain = [&]() {
        Flow* r0 = flow::Intern(a, "s3://1000genomes/technical/reference/human_g1k_v37.fasta.gz");
        r0->Done = true;
        r0->Value = one(id_of(1, 0));
        Flow* r1 = exec("biocontainers/bwa", "\n\tgunzip -c %s > %s/g1k_v37.fa\n\tbwa index -a bwtsw g1k_v37.fa\n",
                        {r0}, id_of(2, 0));
        return op1(OpCoerce, r1, fd_out, r1->Value);
    };
    Flow* r2 = ref_chain();
    std::vector<Flow*> roots;
    std::vector<Digest> files;
    char buf[256];
    for (uint64_t s = 0; s < S; ++s) {
        if (dup && s) r2 = ref_chain();
        std::vector<Flow*> bams;
        for (uint64_t p = 0; p < P; ++p) {
            const uint64_t q = s * P + p;
            Flow* v[2];
            for (int k = 0; k < 2; ++k) {
                files.push_back(id_of(3, 2 * q + k));
                v[k] = op1(OpCoerce, flow::Val(a, one(files.back())), fd_coerce, one(files.back()));
            }
            snprintf(buf, sizeof buf, "\n\t\tbwa mem -R \"@RG\\tID:S%07llu_P%03llu\\tSM:S%07llu\" -t 32 \\\n"
                                      "\t\t\t%%s/g1k_v37.fa %%s %%s > %%s\n\t",
                     (unsigned long long)s, (unsigned long long)p, (unsigned long long)s);
            Flow* e1 = exec("biocontainers/bwa", buf, {r2, v[0], v[1]}, id_of(4, q));
            Flow* k1 = op1(OpCoerce, op1(OpK, op1(OpCoerce, e1, fd_out, e1->Value), fd_force, e1->Value), fd_fs, e1->Value);
            snprintf(buf, sizeof buf, "\n\t\t< %%s samtools view -Sb - > %%s # S%07llu_P%03llu\n\t",
                     (unsigned long long)s, (unsigned long long)p);
            Flow* e2 = exec("biocontainers/samtools", buf, {k1}, id_of(5, q));
            Flow* k2 = op1(OpCoerce, op1(OpK, op1(OpCoerce, e2, fd_out, e2->Value), fd_force, e2->Value), fd_fs, e2->Value);
            snprintf(buf, sizeof buf, "\n\t\tsamtools sort --threads 64 -o %%s %%s # S%07llu_P%03llu\n\t",
                     (unsigned long long)s, (unsigned long long)p);
            Flow* e3 = exec("biocontainers/samtools", buf, {k2}, id_of(6, q));
            bams.push_back(op1(OpCoerce, e3, fd_out, e3->Value));
        }
        Fileset lst;
        lst.List = std::vector<Fileset>{};
        for (Flow* b : bams) lst.List->push_back(*b->Value);
        Flow ks;
        ks.op = OpK;
        ks.Deps = bams;
        ks.FlowDigest = fd_merge;
        ks.Done = true;
        ks.Value = lst;
        Flow* cs1 = op1(OpCoerce, a.New(std::move(ks)), fd_fs, lst);
        snprintf(buf, sizeof buf, "\n\t\tsamtools merge -@64 %%s %%s # S%07llu\n\t", (unsigned long long)s);
        Flow* es = exec("biocontainers/samtools", buf, {cs1}, id_of(7, s));
        snprintf(buf, sizeof buf, "s3://1000genomes-out/S%07llu.bam", (unsigned long long)s);
        roots.push_back(flow::Extern(a, buf, op1(OpCoerce, es, fd_out, es->Value)));
    }
    Flow* top = flow::Merge(a, roots);
    if (copyprobe) return copy_probe(top, (unsigned)(argc > 4 ? atoi(argv[4]) : 8));
    Engine& e = *eng;
    const uint64_t n_nodes = 4 + S * (P * 14 + 6) + (dup && S ? 3 * (S - 1) : 0);
    const double t_build = secs(t0);
    t0 = Clock::now();
    std::unique_ptr<Eval> lowered;
    Flow* c = Canonicalize(e, a, top, Config{false}, "", &lowered);
    const double t_canon = secs(t0);
    // Canonicalize hands over its Eval (the canonical graph's, loaded and
    // recomputed; collapsed copies' jobs dropped)
    const bool handed_over = lowered != nullptr;
    double t_lower = 0, t_load = 0;
    if (!lowered) {
        lowered = std::make_unique<Eval>(e, "", true);
        t0 = Clock::now();
        lowered->Add(c);
        t_lower = secs(t0);
        t0 = Clock::now();
        lowered->Build();
        t_load = secs(t0);
    }
    Eval& ev = *lowered;
    // 1% of the File IDs replaced, one SetFileID each (the shim's per-file call)
    t0 = Clock::now();
    const uint64_t nf = files.size(), nch = nf / 100;
    for (uint64_t k = 0; k < nch; ++k) {
        const uint64_t i = (k * 7919) % nf;
        Digest nw = id_of(8, i);
        ev.SetFileID(files[i], nw);
        files[i] = nw;
    }
    const double t_set = secs(t0);
    t0 = Clock::now();
    const uint64_t hashed = ev.Recompute(false);
    const double t_inc = secs(t0);
    const Digest inc_root = ev.FlowDigest(c);
    const std::vector<Digest> inc_keys = ev.CacheKeys(c->Deps.front());
    ev.Recompute(true);
    const bool same = ev.FlowDigest(c) == inc_root && ev.CacheKeys(c->Deps.front()) == inc_keys;
    printf("{\"samples\": %llu, \"pairs\": %llu, \"nodes\": %llu, \"jobs\": %zu, \"build_s\": %.3f, "
           "\"canonicalize_s\": %.3f, \"lower_s\": %.3f, \"load_s\": %.3f, \"set_file_ids_s\": %.3f, "
           "\"files_changed\": %llu, \"incremental_s\": %.4f, \"jobs_rehashed\": %llu, "
           "\"incremental_equals_full\": %s, \"canonicalize_handed_over\": %s, \"collapsed\": %zu, "
           "\"dup_ref_chains\": %s, \"lower_threads\": %d, \"root\": \"%s\"}\n",
           (unsigned long long)S, (unsigned long long)P, (unsigned long long)n_nodes, ev.Jobs(), t_build, t_canon,
           t_lower, t_load, t_set, (unsigned long long)nch, t_inc, (unsigned long long)hashed, same ? "true" : "false",
           handed_over ? "true" : "false", ev.Collapsed(), dup ? "true" : "false", lower_threads_in_use(e),
           inc_root.String().c_str());
    return same ? 0 : 1;
}

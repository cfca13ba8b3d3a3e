// reflow_host.cpp -- C++ host-side mirror of Reflow's memoization API
// (include/reflow_host.hpp) over the C-ABI.  Lowering follows the byte grammar
// of flow.go:675-792 / executor.go:214-233; every SHA-256 is
// computed by the device through rf_graph_* / rf_sha256_batch /
// rf_fileset_digest_batch.
#include "diag.h"
#include "reflow_host.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <exception>
#include <thread>
#include <mutex>
#include <sys/mman.h>
#include <atomic>
#include <functional>
#include <memory>
#include <unordered_set>

namespace reflow {

namespace detail {
void* huge_page_alloc(size_t bytes) {
    constexpr size_t kHuge = 2u << 20;
    if (bytes < 2 * kHuge) {
        void* p = ::operator new(bytes);
        return p;
    }
    void* p = nullptr;
    if (posix_memalign(&p, kHuge, bytes) != 0) throw std::bad_alloc();
    (void)madvise(p, bytes, MADV_HUGEPAGE);  // (advice only: plain pages if declined)
    return p;
}
void huge_page_free(void* p, size_t bytes) noexcept {
    if (bytes < 2 * (2u << 20))
        ::operator delete(p);
    else
        free(p);
}
}  // namespace detail

void Check(int rc) {
    if (rc != RF_OK) throw Error(rc, rf_last_error());
}

// ---- Digest -----------------------------------------------------------------
bool Digest::IsZero() const {
    for (uint8_t x : b)
        if (x) return false;
    return true;
}

std::string Digest::Hex() const {
    static const char* hx = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; ++i) {
        s[2 * i] = hx[b[i] >> 4];
        s[2 * i + 1] = hx[b[i] & 15];
    }
    return s;
}

std::string Digest::String() const { return "sha256:" + Hex(); }
std::string Digest::Short() const { return "sha256:" + Hex().substr(0, 8); }

bool Digest::Parse(const std::string& s, Digest* out) {
    if (s.size() != 7 + 64 || s.compare(0, 7, "sha256:") != 0) return false;
    auto nib = [](char c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        return -1;
    };
    for (int i = 0; i < 32; ++i) {
        const int hi = nib(s[7 + 2 * i]), lo = nib(s[8 + 2 * i]);
        if (hi < 0 || lo < 0) return false;
        out->b[i] = (uint8_t)(hi << 4 | lo);
    }
    return true;
}

void WriteDigest(std::string& w, const Digest& d) {
    w.push_back('\0');
    w.push_back('\5');
    w.append(reinterpret_cast<const char*>(d.b.data()), 32);
}

// ---- Engine / Digester -----------------------------------------------------
Engine::Engine(int device) { Check(rf_init(device, &ctx_)); }
Engine::~Engine() { rf_destroy(ctx_); }

std::vector<Digest> Digester::FromBytesBatch(const std::vector<std::string>& msgs) {
    std::vector<const uint8_t*> p(msgs.size());
    std::vector<uint64_t> n(msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i) {
        p[i] = reinterpret_cast<const uint8_t*>(msgs[i].data());
        n[i] = msgs[i].size();
    }
    std::vector<Digest> out(msgs.size());
    if (!msgs.empty())
        Check(rf_sha256_batch(e_.ctx(), p.data(), n.data(), msgs.size(), out[0].b.data()));
    return out;
}

// ---- Fileset ------------------------------------------------------------------
void Fileset::WriteDigest(std::string& w) const {
    if (List) {
        for (const Fileset& v : *List) v.WriteDigest(w);
        return;
    }
    for (const auto& [path, file] : Map) {  // std::map: bytewise order == sort.Strings
        w += path;
        reflow::WriteDigest(w, file.ID);
    }
}

size_t Fileset::N() const {
    size_t n = Map.size();
    if (List)
        for (const Fileset& v : *List) n += v.N();
    return n;
}

bool Fileset::Empty() const {
    if (List)
        for (const Fileset& v : *List)
            if (!v.Empty()) return false;
    return Map.empty();
}

std::vector<Digest> FilesetDigests(Engine& e, const std::vector<const Fileset*>& v) {
    std::vector<uint64_t> set_group{0}, group_entry{0};
    std::vector<const char*> paths;
    std::vector<uint32_t> plen;
    std::vector<uint8_t> ids;
    std::function<void(const Fileset&)> groups = [&](const Fileset& f) {
        if (f.List) {
            for (const Fileset& c : *f.List) groups(c);
            return;
        }
        for (const auto& [path, file] : f.Map) {
            paths.push_back(path.data());
            plen.push_back((uint32_t)path.size());
            ids.insert(ids.end(), file.ID.b.begin(), file.ID.b.end());
        }
        group_entry.push_back(paths.size());
    };
    for (const Fileset* f : v) {
        groups(*f);
        set_group.push_back(group_entry.size() - 1);
    }
    std::vector<Digest> out(v.size());
    if (!v.empty())
        Check(rf_fileset_digest_batch(e.ctx(), v.size(), set_group.data(), group_entry.data(),
                                      paths.data(), plen.data(), ids.data(), out[0].b.data()));
    return out;
}

Fileset Install(Engine& e, const std::string& path, Digest* digest) {
    rf_install* in = nullptr;
    Check(rf_install_dir(e.ctx(), path.c_str(), &in));
    std::unique_ptr<rf_install, void (*)(rf_install*)> guard(in, rf_install_destroy);
    uint64_t n = 0, pb = 0;
    Digest fs;
    Check(rf_install_info(in, &n, &pb, fs.b.data()));
    std::string paths(pb, '\0');
    std::vector<uint64_t> offs(n + 1);
    std::vector<uint8_t> ids(32 * n);
    std::vector<int64_t> sizes(n);
    Check(rf_install_entries(in, paths.data(), offs.data(), ids.data(), sizes.data()));
    Fileset v;
    for (uint64_t i = 0; i < n; ++i) {
        File f;
        memcpy(f.ID.b.data(), ids.data() + 32 * i, 32);
        f.Size = sizes[i];
        v.Map.emplace(paths.substr(offs[i], offs[i + 1] - offs[i]), f);
    }
    if (digest) *digest = fs;
    return v;
}

// Fileset trees in the rf_fileset_tree CSR form (pre-order nodes; a node's
// Map entries before its children's).
namespace {
struct TreeArrays {
    std::vector<uint64_t> list_ptr{0}, entry_ptr{0};
    std::vector<uint32_t> list_child;
    std::vector<std::vector<uint32_t>> kids;
    std::vector<const char*> paths;
    std::vector<uint32_t> plen;
    std::vector<uint8_t> ids;
    std::vector<int64_t> sizes;
    uint32_t add(const Fileset& f) {
        const uint32_t node = (uint32_t)kids.size();
        kids.emplace_back();
        for (const auto& [path, file] : f.Map) {
            paths.push_back(path.data());
            plen.push_back((uint32_t)path.size());
            ids.insert(ids.end(), file.ID.b.begin(), file.ID.b.end());
            sizes.push_back(file.Size);
        }
        entry_ptr.push_back(paths.size());
        if (f.List)
            for (const Fileset& c : *f.List) {
                const uint32_t k = add(c);
                kids[node].push_back(k);
            }
        return node;
    }
    rf_fileset_tree tree() {
        for (auto& k : kids) {
            list_child.insert(list_child.end(), k.begin(), k.end());
            list_ptr.push_back(list_child.size());
        }
        return rf_fileset_tree{kids.size(), list_ptr.data(), list_child.data(), entry_ptr.data(),
                               paths.data(), plen.data(), ids.data(), sizes.data()};
    }
};
}  // namespace

std::string MarshalJSON(const Fileset& v) {
    TreeArrays a;
    const uint32_t root = a.add(v);
    const rf_fileset_tree t = a.tree();
    uint64_t need = 0;
    if (rf_fileset_marshal_json(&t, root, nullptr, 0, &need) != RF_OK && need == 0) Check(RF_EINVAL);
    std::string out(need, '\0');
    Check(rf_fileset_marshal_json(&t, root, reinterpret_cast<uint8_t*>(out.data()), need, &need));
    return out;
}

std::vector<Digest> FilesetValueDigests(Engine& e, const std::vector<const Fileset*>& v) {
    TreeArrays a;
    std::vector<uint32_t> roots;
    for (const Fileset* f : v) roots.push_back(a.add(*f));
    const rf_fileset_tree t = a.tree();
    std::vector<Digest> out(v.size());
    if (!v.empty()) Check(rf_fileset_value_digest_batch(e.ctx(), &t, roots.data(), roots.size(), out[0].b.data()));
    return out;
}

// ---- flows ----------------------------------------------------------------------
std::string DigestString(Op op) {
    static const char* names[] = {"OpExec", "OpIntern", "OpExtern", "OpGroupby", "OpMap",
                                  "OpCollect", "OpMerge", "OpVal", "OpPullup", "OpK",
                                  "OpCoerce", "OpRequirements", "maxOp"};
    const int i = (int)op - 1;
    if (i < 0 || i >= 13) return "Op(" + std::to_string((int)op) + ")";
    return names[i];
}

namespace flow {
Flow* Exec(FlowArena& a, const std::string& image, const std::string& cmd, std::vector<Flow*> deps) {
    Flow f;
    f.op = OpExec;
    f.Deps = std::move(deps);
    f.Image = image;
    f.Cmd = cmd;
    return a.New(std::move(f));
}
Flow* Intern(FlowArena& a, const std::string& url) {
    Flow f;
    f.op = OpIntern;
    f.URL = url;
    return a.New(std::move(f));
}
Flow* Extern(FlowArena& a, const std::string& url, Flow* dep) {
    Flow f;
    f.op = OpExtern;
    f.URL = url;
    f.Deps = {dep};
    return a.New(std::move(f));
}
Flow* Groupby(FlowArena& a, const std::string& re, Flow* dep) {
    Flow f;
    f.op = OpGroupby;
    f.Re = re;
    f.Deps = {dep};
    return a.New(std::move(f));
}
Flow* Collect(FlowArena& a, const std::string& re, const std::string& repl, Flow* dep) {
    Flow f;
    f.op = OpCollect;
    f.Re = re;
    f.Repl = repl;
    f.Deps = {dep};
    return a.New(std::move(f));
}
Flow* Merge(FlowArena& a, std::vector<Flow*> deps) {
    Flow f;
    f.op = OpMerge;
    f.Deps = std::move(deps);
    return a.New(std::move(f));
}
Flow* Pullup(FlowArena& a, std::vector<Flow*> deps) {
    Flow f;
    f.op = OpPullup;
    f.Deps = std::move(deps);
    return a.New(std::move(f));
}
Flow* Val(FlowArena& a, const Fileset& v) {  // Fileset.Flow: OpVal, FlowDone
    Flow f;
    f.op = OpVal;
    f.Value = v;
    f.Done = true;
    return a.New(std::move(f));
}
Flow* Data(FlowArena& a, const std::string& b) {
    Flow f;
    f.op = OpData;
    f.Data = b;
    return a.New(std::move(f));
}
}  // namespace flow

// ---- Eval: lowering to rf_graph jobs ------------------------------------------
static void writeN(std::string& w, int64_t n) {
    const uint64_t u = (uint64_t)n;
    for (int i = 0; i < 8; ++i) w.push_back((char)(u >> (8 * i)));
}

static void exec_suffix(const Flow* f, std::string& w) {
    w += f->Image;
    w += f->Cmd;
    if (f->Argmap)
        for (const ExecArg& a : *f->Argmap) writeN(w, a.Out ? -(int64_t)a.Index : a.Index);
}

// op names without a string allocation per node (DigestString's table)
static void append_op_name(std::string& w, Op op) {
    static const char* names[] = {"OpExec", "OpIntern", "OpExtern", "OpGroupby", "OpMap",
                                  "OpCollect", "OpMerge", "OpVal", "OpPullup", "OpK",
                                  "OpCoerce", "OpRequirements", "maxOp"};
    const int i = (int)op - 1;
    if (i < 0 || i >= 13)
        w += DigestString(op);
    else
        w += names[i];
}

// Host threads for the lowering: the engine's host-leg width (the process's
// CPU share, min(60, share) / ranks per node), at least 1; RF_LOWER_THREADS
// overrides.
static unsigned lower_threads(Engine& e) {
    if (const char* v = getenv("RF_LOWER_THREADS")) return std::max(1, atoi(v));
    int th = 0, ext = 0;
    double rate = 0;
    if (rf_host_info(e.ctx(), &th, &rate, &ext) != RF_OK || th < 1) {
        const unsigned h = std::thread::hardware_concurrency();
        th = (int)std::min(h ? h : 1u, 16u);
    }
    return (unsigned)th;
}

// RF_LOWER_TIMING=1: phase times of the lowering on stderr
static bool lower_timing() {
    static const bool on = getenv("RF_LOWER_TIMING") != nullptr;
    return on;
}
struct PhaseClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!lower_timing()) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[lower] %s %.3f s\n", what, std::chrono::duration<double>(now - t).count());
        t = now;
    }
};

// Ranges [lo, hi) of n items of `grain` each, claimed by `threads` threads;
// fn(range index, lo, hi).  The first exception a worker throws is rethrown.
template <class F>
static void parallel_ranges(size_t n, size_t grain, unsigned threads, F fn) {
    const size_t nr = (n + grain - 1) / grain;
    if (nr <= 1 || threads <= 1) {
        for (size_t r = 0; r < nr; ++r) fn(r, r * grain, std::min(n, (r + 1) * grain));
        return;
    }
    std::atomic<size_t> next{0};
    std::exception_ptr err;
    std::mutex mu;
    auto work = [&]() {
        try {
            for (size_t r; (r = next.fetch_add(1)) < nr;) fn(r, r * grain, std::min(n, (r + 1) * grain));
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
            next.store(nr);
        }
    };
    std::vector<std::thread> th;
    const unsigned t = (unsigned)std::min<size_t>(threads, nr);
    for (unsigned i = 1; i < t; ++i) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    if (err) std::rethrow_exception(err);
}

Eval::Eval(Engine& e, std::string universe, bool file_slots)
    : e_(e), U_(std::move(universe)), file_slots_(file_slots) {}

Eval::~Eval() {
    if (g_) rf_graph_destroy(g_);
}

const uint32_t* Eval::slot_of(const Flow* f) const {
    for (const Block& b : blocks_)
        if (f >= b.base && f < b.base + b.n) {
            // (a static per thread: the slot is returned by pointer like the map's)
            thread_local uint32_t s;
            s = b.slot0 + (uint32_t)b.at(f);
            return &s;
        }
    return logical_.find(f);
}

const uint32_t* Eval::phys_slot_of(const Flow* f) const {
    for (const Block& b : blocks_)
        if (f >= b.base && f < b.base + b.n) {
            const uint32_t* s = &b.phys[b.at(f)];
            return *s == ~0u ? nullptr : s;
        }
    return physical_.find(f);
}

// With file slots, a File ID becomes a hole whose slot is given after the
// parallel phase (one slot per distinct ID); else WD(ID) inline.
void Eval::fileset_material(const Fileset& v, std::string& out, Holes& holes, FileRefs& files) const {
    if (v.List) {
        for (const Fileset& c : *v.List) fileset_material(c, out, holes, files);
        return;
    }
    for (const auto& [path, file] : v.Map) {
        out += path;
        if (file_slots_) {
            out.push_back('\0');
            out.push_back('\5');
            files.emplace_back((uint32_t)holes.size(), file.ID);
            holes.emplace_back((uint32_t)out.size(), 0u);
            out.append(32, '\0');
        } else {
            WriteDigest(out, file.ID);
        }
    }
}

// Flow.WriteDigest (flow.go:675-750) with WD(dep.Digest()) as holes.  Each
// node's own Config.HashV1 decides whether its deps are inlined (flow.go:
// 692-697); an inlined dep follows its own config in turn, and so does a
// Parent (Canonicalize merges the config into the copies it makes, never
// into f.Parent: flow.go:818-843).  Every dep already has its slot (the
// nodes are numbered before any material is built), so this only reads.
void Eval::material(const Flow* f, std::string& out, Holes& holes, FileRefs& files) const {
    out += U_;
    if (f->op == OpRequirements) {
        material(f->Deps.at(0), out, holes, files);
        return;
    }
    if (f->Parent) {
        material(f->Parent, out, holes, files);
        return;
    }
    for (const Flow* d : f->Deps) {
        if (f->config.HashV1) {
            material(d, out, holes, files);
        } else {
            const uint32_t* s = slot_of(d);
            if (!s) throw Error(RF_EINVAL, "dependency not numbered (a Flow reachable only after Add)");
            out.push_back('\0');
            out.push_back('\5');
            holes.emplace_back((uint32_t)out.size(), *s);
            out.append(32, '\0');
        }
    }
    append_op_name(out, f->op);
    switch (f->op) {
    case OpIntern:
    case OpExtern: out += f->URL; break;
    case OpExec: exec_suffix(f, out); break;
    case OpGroupby: out += f->Re; break;
    case OpMap: material(f->MapFlow, out, holes, files); break;
    case OpCollect: out += f->Re; out += f->Repl; break;
    case OpVal:
        if (f->Err) throw Error(RF_EINVAL, "error OpVal digests are random (flow.go:722-731)");
        if (f->Value) {
            fileset_material(*f->Value, out, holes, files);
        } else {
            if (f->FlowDigest.IsZero()) throw Error(RF_EINVAL, "invalid flow digest");
            WriteDigest(out, f->FlowDigest);
        }
        break;
    case OpK:
    case OpCoerce:
        if (f->FlowDigest.IsZero()) throw Error(RF_EINVAL, "invalid flow digest");
        WriteDigest(out, f->FlowDigest);
        break;
    case OpData: out += f->Data; break;
    default: break;  // OpMerge, OpPullup
    }
}

// Flow.PhysicalDigest (flow.go:764-792) exists for OpExec / OpExtern whose
// deps are all FlowDone: no Universe, no op name, no WD.
static bool has_physical(const Flow* f) {
    if (f->op != OpExec && f->op != OpExtern) return false;
    for (const Flow* d : f->Deps)
        if (!d->Done) return false;
    return true;
}

struct Eval::Part {
    std::string blob;
    std::vector<uint32_t> out_slot, tmpl_len, hole_pos, hole_slot;
    std::vector<uint64_t> tmpl_off, hole_end;     // per job: local template offset, local hole end
    std::vector<std::pair<uint64_t, Digest>> files;  // (local hole index, File ID)
};

// The logical (and physical) jobs of nodes -- `nodes`, or every node of
// `blk` -- whose slots are all given: materials built on host threads, one
// part per range of nodes, then the File IDs' slots (in part order, so the
// numbering is deterministic) and the parts appended in order.
void Eval::lower_nodes(const std::vector<const Flow*>* nodes, const Block* blk, const std::vector<uint32_t>& phys) {
    const size_t n = nodes ? nodes->size() : blk->n;
    PhaseClock pc;
    constexpr size_t kGrain = 8192;
    std::vector<Part> parts((n + kGrain - 1) / kGrain);
    parallel_ranges(n, kGrain, lower_threads(e_), [&](size_t r, size_t lo, size_t hi) {
        Part& P = parts[r];
        std::string t;
        Holes h;
        FileRefs files;
        auto commit = [&](uint32_t out) {
            P.out_slot.push_back(out);
            P.tmpl_off.push_back(P.blob.size());
            P.tmpl_len.push_back((uint32_t)t.size());
            P.blob += t;
            for (const auto& [hi_, d] : files) P.files.emplace_back(P.hole_pos.size() + hi_, d);
            for (const auto& [pos, slot] : h) {
                P.hole_pos.push_back(pos);
                P.hole_slot.push_back(slot);
            }
            P.hole_end.push_back(P.hole_pos.size());
        };
        for (size_t i = lo; i < hi; ++i) {
            const Flow* f = nodes ? (*nodes)[i] : blk->base + i;
            t.clear();
            h.clear();
            files.clear();
            material(f, t, h, files);
            commit(nodes ? *slot_of(f) : blk->slot0 + (uint32_t)i);
            if (phys[i] != ~0u) {
                t.clear();
                h.clear();
                files.clear();
                for (const Flow* d : f->Deps) {
                    if (!d->Value) throw Error(RF_EINVAL, "done dependency without a Fileset value");
                    fileset_material(*d->Value, t, h, files);
                }
                if (f->op == OpExtern)
                    t += f->URL;
                else
                    exec_suffix(f, t);
                commit(phys[i]);
            }
        }
    });
    pc.lap("materials (threads)");
    const unsigned th = lower_threads(e_);
    // File IDs: one slot per distinct ID, resolved shard by shard on host
    // threads.  A new ID gets a provisional shard-local number (bit 31), and
    // after every shard is done the final slots follow shard by shard, first
    // occurrence in part order within a shard: deterministic.
    constexpr uint32_t kProv = 0x80000000u;
    if (n_slots_ & kProv) throw Error(RF_EINVAL, "too many slots");
    std::vector<uint64_t> ref0(parts.size() + 1, 0);
    for (size_t r = 0; r < parts.size(); ++r) ref0[r + 1] = ref0[r] + parts[r].files.size();
    std::vector<uint32_t> ref_val(ref0.back());
    std::vector<uint32_t> new_in(kFileShards, 0);
    parallel_ranges(kFileShards, 1, th, [&](size_t sh, size_t, size_t) {
        auto& m = file_slot_[sh];
        uint32_t fresh = 0;
        for (size_t r = 0; r < parts.size(); ++r) {
            const auto& F = parts[r].files;
            for (size_t k = 0; k < F.size(); ++k) {
                if (file_shard(F[k].second) != sh) continue;
                uint32_t v;
                if (const uint32_t* q = m.find(F[k].second)) {
                    v = *q;
                } else {
                    v = kProv | fresh++;
                    m.insert(F[k].second, v);
                }
                ref_val[ref0[r] + k] = v;
            }
        }
        new_in[sh] = fresh;
    });
    pc.lap("file refs (threads)");
    std::vector<uint32_t> sbase(kFileShards);
    for (unsigned sh = 0; sh < kFileShards; ++sh) {
        sbase[sh] = n_slots_;
        n_slots_ += new_in[sh];
        if (n_slots_ & kProv) throw Error(RF_EINVAL, "too many slots");
    }
    parallel_ranges(kFileShards, 1, th, [&](size_t sh, size_t, size_t) {
        if (new_in[sh])
            file_slot_[sh].for_each_mut([&](const Digest&, uint32_t& v) {
                if (v & kProv) v = sbase[sh] + (v & ~kProv);
            });
    });
    pc.lap("file slots final");
    // the parts appended in order (offsets first, then copied on host threads)
    const size_t J0 = out_slot_.size(), H0 = hole_pos_.size(), B0 = blob_.size();
    std::vector<size_t> pj(parts.size() + 1, J0), ph(parts.size() + 1, H0), pb(parts.size() + 1, B0);
    for (size_t r = 0; r < parts.size(); ++r) {
        pj[r + 1] = pj[r] + parts[r].out_slot.size();
        ph[r + 1] = ph[r] + parts[r].hole_pos.size();
        pb[r + 1] = pb[r] + parts[r].blob.size();
    }
    out_slot_.resize(pj.back());
    tmpl_off_.resize(pj.back());
    tmpl_len_.resize(pj.back());
    hole_ptr_.resize(pj.back() + 1);
    hole_pos_.resize(ph.back());
    hole_slot_.resize(ph.back());
    blob_.resize(pb.back());
    pc.lap("resize");
    parallel_ranges(parts.size(), 1, th, [&](size_t r, size_t, size_t) {
        Part& P = parts[r];
        for (size_t k = 0; k < P.files.size(); ++k) {
            const uint32_t v = ref_val[ref0[r] + k];
            P.hole_slot[P.files[k].first] = (v & kProv) ? sbase[file_shard(P.files[k].second)] + (v & ~kProv) : v;
        }
        memcpy(&blob_[pb[r]], P.blob.data(), P.blob.size());
        std::copy(P.out_slot.begin(), P.out_slot.end(), out_slot_.begin() + pj[r]);
        std::copy(P.tmpl_len.begin(), P.tmpl_len.end(), tmpl_len_.begin() + pj[r]);
        for (size_t k = 0; k < P.tmpl_off.size(); ++k) {
            tmpl_off_[pj[r] + k] = pb[r] + P.tmpl_off[k];
            hole_ptr_[pj[r] + k + 1] = ph[r] + P.hole_end[k];
        }
        std::copy(P.hole_pos.begin(), P.hole_pos.end(), hole_pos_.begin() + ph[r]);
        std::copy(P.hole_slot.begin(), P.hole_slot.end(), hole_slot_.begin() + ph[r]);
        Part().blob.swap(P.blob);
    });
    pc.lap("append (threads)");
}

// Every node reachable through Deps, MapFlow and Parent that this Eval has
// not lowered yet: numbered first (logical slot, physical slot), then lowered
// on host threads (lower_nodes).
void Eval::Add(Flow* root) {
    PhaseClock pc;
    std::vector<const Flow*> todo;
    std::vector<const Flow*> stack{root};
    while (!stack.empty()) {
        const Flow* f = stack.back();
        stack.pop_back();
        if (!f || slot_of(f)) continue;
        logical_.insert(f, new_slot());
        todo.push_back(f);
        for (const Flow* d : f->Deps) stack.push_back(d);
        if (f->MapFlow) stack.push_back(f->MapFlow);
        if (f->Parent) stack.push_back(f->Parent);
    }
    std::vector<uint32_t> phys(todo.size(), ~0u);
    for (size_t i = 0; i < todo.size(); ++i)
        if (has_physical(todo[i]) && !physical_.find(todo[i])) {
            phys[i] = new_slot();
            physical_.insert(todo[i], phys[i]);
        }
    pc.lap("numbering");
    lower_nodes(&todo, nullptr, phys);
}

// A contiguous run of nodes whose deps and map flows lie in the run (or were
// added before): slots by address.  Nodes reachable only through a Parent
// outside the run take the general path afterwards.
void Eval::add_block(const Flow* base, size_t n) {
    Block b{base, n, n_slots_, std::vector<uint32_t>(n, ~0u)};
    n_slots_ += (uint32_t)n;
    for (size_t i = 0; i < n; ++i)
        if (has_physical(base + i)) b.phys[i] = new_slot();
    blocks_.push_back(std::move(b));
    const Block& blk = blocks_.back();
    std::vector<const Flow*> parents;
    for (size_t i = 0; i < n; ++i)
        if (base[i].Parent && !slot_of(base[i].Parent)) parents.push_back(base[i].Parent);
    // the run's own deps must be numbered before its materials are built
    for (const Flow* p : parents) Add(const_cast<Flow*>(p));
    lower_nodes(nullptr, &blk, blk.phys);
}

void Eval::Build() {
    PhaseClock pc;
    load();
    pc.lap("build: rf_graph_load");
    if (const size_t nf = n_files()) {
        // every File ID into its slot, the shards gathered on host threads
        detail::RawVec<uint32_t> s(nf);
        detail::RawVec<uint8_t> ids(32 * nf);
        std::vector<size_t> at(kFileShards + 1, 0);
        for (unsigned sh = 0; sh < kFileShards; ++sh) at[sh + 1] = at[sh] + file_slot_[sh].size();
        parallel_ranges(kFileShards, 1, lower_threads(e_), [&](size_t sh, size_t, size_t) {
            size_t k = at[sh];
            file_slot_[sh].for_each([&](const Digest& id, uint32_t slot) {
                s[k] = slot;
                memcpy(&ids[32 * k], id.b.data(), 32);
                ++k;
            });
        });
        Check(rf_graph_set_slots(g_, s.data(), ids.data(), (uint32_t)nf));
        pc.lap("build: file IDs set");
    }
    Recompute(true);
    pc.lap("build: full recompute");
}

// The job arrays onto the device (rf_graph_load), replacing any graph loaded before.
void Eval::load() {
    const uint32_t J = (uint32_t)out_slot_.size();
    rf_graph_desc d{J,
                    n_slots_,
                    out_slot_.data(),
                    tmpl_off_.data(),
                    tmpl_len_.data(),
                    hole_ptr_.data(),
                    hole_pos_.empty() ? nullptr : hole_pos_.data(),
                    hole_slot_.empty() ? nullptr : hole_slot_.data(),
                    reinterpret_cast<const uint8_t*>(blob_.data()),
                    blob_.size()};
    if (g_) rf_graph_destroy(g_);
    g_ = nullptr;
    Check(rf_graph_load(e_.ctx(), &d, &g_));
}

uint64_t Eval::Recompute(bool full) {
    uint64_t n = 0;
    Check(rf_graph_recompute(g_, full ? 1 : 0, &n));
    cache_ok_ = false;
    return n;
}

void Eval::fetch() const {
    if (cache_ok_) return;
    std::vector<uint32_t> idx(n_slots_);
    for (uint32_t i = 0; i < n_slots_; ++i) idx[i] = i;
    cache_.assign(32ull * n_slots_, 0);
    if (n_slots_) Check(rf_graph_get_slots(g_, idx.data(), n_slots_, cache_.data()));
    cache_ok_ = true;
}

Digest Eval::FlowDigest(const Flow* f) const {
    fetch();
    const uint32_t* s = slot_of(f);
    if (!s) throw Error(RF_ENOTFOUND, "flow not in this Eval");
    Digest d;
    memcpy(d.b.data(), cache_.data() + 32ull * *s, 32);
    return d;
}

std::optional<Digest> Eval::PhysicalDigest(const Flow* f) const {
    const uint32_t* s = phys_slot_of(f);
    if (!s) return std::nullopt;
    fetch();
    Digest d;
    memcpy(d.b.data(), cache_.data() + 32ull * *s, 32);
    return d;
}

// CacheKeys (flow.go:796-802): most to least concrete.
std::vector<Digest> Eval::CacheKeys(const Flow* f) const {
    std::vector<Digest> keys;
    if (auto p = PhysicalDigest(f)) keys.push_back(*p);
    keys.push_back(FlowDigest(f));
    return keys;
}

void Eval::SetFileID(const Digest& old_id, const Digest& new_id) {
    auto& mo = file_slot_[file_shard(old_id)];
    const uint32_t* p = mo.find(old_id);
    if (!p) throw Error(RF_ENOTFOUND, "file id not referenced: " + old_id.String());
    const uint32_t s = *p;
    mo.erase(old_id);
    auto& mn = file_slot_[file_shard(new_id)];
    if (uint32_t* q = mn.find(new_id))
        *q = s;  // (an ID already in use elsewhere: the map keeps the last slot, as before)
    else
        mn.insert(new_id, s);
    Check(rf_graph_set_slots(g_, &s, new_id.b.data(), 1));
}

// ---- Canonicalize ------------------------------------------------------------
namespace detail {
// (reflow_host.hpp)
void PostOrder(Flow* root, unsigned threads, std::vector<Flow*>& post, PtrIndex& index) {
    using Index = PtrIndex;
    struct Frame {
        Flow* f;
        size_t next;  // next dep (then MapFlow) to visit
    };
    // the post-order from `start`, skipping (and marking) what `seen` holds
    auto dfs = [](Flow* start, Index& seen, std::vector<Flow*>& out) {
        std::vector<Frame> st{{start, 0}};
        while (!st.empty()) {
            Frame& fr = st.back();
            Flow* f = fr.f;
            const size_t nd = f->Deps.size() + (f->MapFlow ? 1 : 0);
            if (fr.next == 0)  // (first visit: the deps' index slots and records on their way in)
                for (Flow* d : f->Deps) {
                    seen.prefetch(d);
                    __builtin_prefetch(d);
                }
            if (fr.next < nd) {
                Flow* d = fr.next < f->Deps.size() ? f->Deps[fr.next] : f->MapFlow;
                ++fr.next;
                if (!seen.find(d)) st.push_back(Frame{d, 0});
                continue;
            }
            st.pop_back();
            if (seen.find(f)) continue;  // reached twice before its first visit completed
            seen.insert(f, (uint32_t)out.size());
            out.push_back(f);
        }
    };
    index.reserve(1u << 16);
    post.clear();
    const size_t nkids = root->Deps.size() + (root->MapFlow ? 1 : 0);
    const unsigned lt = threads;
    if (nkids >= 256 && lt > 1) {
        // A wide root (1000align: one dep per sample): the root's children in
        // contiguous groups, each group's post-order on a host thread with a
        // visited set of its own, then the groups concatenated in order with
        // what an earlier group already emitted dropped.  That is the
        // sequential order exactly: a DFS that finds a node already visited
        // skips its whole subtree, and everything below a visited node was
        // visited with it, so group g's walk with the earlier groups' nodes
        // pre-visited emits its own walk's order minus those nodes.
        auto kid = [&](size_t i) { return i < root->Deps.size() ? root->Deps[i] : root->MapFlow; };
        const size_t ng = std::min<size_t>(nkids, 8ull * lt);
        std::vector<std::vector<Flow*>> part(ng);
        parallel_ranges(ng, 1, lt, [&](size_t r, size_t, size_t) {
            Index seen;
            seen.reserve(1u << 12);
            for (size_t i = r * nkids / ng; i < (r + 1) * nkids / ng; ++i)
                if (!seen.find(kid(i))) dfs(kid(i), seen, part[r]);
        });
        size_t total = 1;
        for (const auto& v : part) total += v.size();
        index.reserve(total);
        post.reserve(total);
        for (auto& v : part) {
            for (size_t k = 0; k < v.size(); ++k) {
                if (k + 16 < v.size()) index.prefetch(v[k + 16]);  // (a miss per lookup otherwise)
                if (!index.find(v[k])) {
                    index.insert(v[k], (uint32_t)post.size());
                    post.push_back(v[k]);
                }
            }
            std::vector<Flow*>().swap(v);
        }
        if (!index.find(root)) {
            index.insert(root, (uint32_t)post.size());
            post.push_back(root);
        }
        if (RF_DIAG_KNOB("RF_LOWER_CHECK_ORDER", 0)) {  // diagnostic build: the sequential walk, compared node for node
            Index seen;
            std::vector<Flow*> seq;
            dfs(root, seen, seq);
            if (seq != post) throw std::runtime_error("Canonicalize: parallel post-order differs from the sequential one");
            fprintf(stderr, "[lower] canonicalize: parallel post-order == sequential (%zu nodes)\n", seq.size());
        }
    } else {
        dfs(root, index, post);
    }
}
}  // namespace detail

Flow* Canonicalize(Engine& e, FlowArena& arena, Flow* root, Config config, const std::string& U,
                   std::unique_ptr<Eval>* lowered) {
    if (lowered) lowered->reset();
    PhaseClock pc;
    // 1. the originals reachable through Deps and MapFlow in post-order (deps,
    //    then the map flow, then the node: the order of flowMap.Put,
    //    flow.go:820-839); each one's index in it.
    detail::PtrIndex index;
    std::vector<Flow*> post;
    detail::PostOrder(root, lower_threads(e), post, index);
    const size_t n = post.size();
    pc.lap("canonicalize: post-order");
    // 2. one copy per original, contiguous in post-order (f.Copy() +
    //    Config.Merge, deps and map flow pointing at copies), on host threads
    Flow* cp = arena.NewN(n, [&](Flow* blk, size_t, size_t) {
        // copy-constructed in place on host threads (a node's deps and map
        // flow point at copies by their post-order index; copies that a
        // thread already made are never touched by another).  A failing
        // range's constructed nodes are destroyed by parallel_ranges'
        // rethrow path below, so none survive an exception.
        std::vector<std::pair<size_t, size_t>> done;
        std::mutex mu;
        try {
            parallel_ranges(n, 16384, lower_threads(e), [&](size_t, size_t lo, size_t hi) {
                size_t i = lo;
                try {
                    for (; i < hi; ++i) {
                        Flow* c = new (blk + i) Flow(*post[i]);
                        c->config.Merge(config);
                        for (Flow*& d : c->Deps) d = blk + *index.find(d);
                        if (c->MapFlow) c->MapFlow = blk + *index.find(c->MapFlow);
                    }
                } catch (...) {
                    for (size_t k = lo; k < i; ++k) blk[k].~Flow();
                    throw;
                }
                std::lock_guard<std::mutex> lk(mu);
                done.emplace_back(lo, hi);
            });
        } catch (...) {
            for (auto& r : done)
                for (size_t k = r.first; k < r.second; ++k) blk[k].~Flow();
            throw;
        }
    });
    pc.lap("canonicalize: copies (threads)");
    // 3. digests of every copy on the device: copy i in slot i
    auto ev = std::make_unique<Eval>(e, U, true);
    ev->add_block(cp, n);
    pc.lap("canonicalize: lowered");
    ev->Build();
    pc.lap("canonicalize: load + full recompute");
    // 4. flowMap.Put: first copy with a digest wins (K5 on the device: the
    //    smallest post-order index of each digest class) -- the copies'
    //    digests are slots [0, n) in post-order, gathered from the slot table
    //    on the device (no round trip of the table through the host)
    std::vector<uint32_t> first(n);
    uint32_t n_unique = 0;
    if (n) {
        struct Dev {
            rf_ctx* c;
            void* p = nullptr;
            ~Dev() {
                if (p) rf_free(c, p);
            }
        } idx{e.ctx()}, dig{e.ctx()}, canon{e.ctx()}, nu{e.ctx()};
        std::vector<uint32_t> iota(n);
        for (size_t i = 0; i < n; ++i) iota[i] = ev->blocks_.front().slot0 + (uint32_t)i;
        Check(rf_malloc(e.ctx(), 4ull * n, &idx.p));
        Check(rf_malloc(e.ctx(), 32ull * n, &dig.p));
        Check(rf_malloc(e.ctx(), 4ull * n, &canon.p));
        Check(rf_malloc(e.ctx(), 64, &nu.p));
        Check(rf_memcpy_h2d(e.ctx(), idx.p, iota.data(), 4ull * n));
        void* st = rf_stream(e.ctx());
        Check(rf_graph_gather_device(ev->g_, idx.p, (uint32_t)n, dig.p, st));
        Check(rf_dedup_digests_device(e.ctx(), dig.p, (uint32_t)n, canon.p, nu.p, st));
        Check(rf_memcpy_d2h(e.ctx(), first.data(), canon.p, 4ull * n));
        Check(rf_memcpy_d2h(e.ctx(), &n_unique, nu.p, 4));
        if (n_unique & 0x80000000u) throw Error(RF_EDEVICE, "canonicalize: dedup probe bound reached");
    }
    pc.lap("canonicalize: dedup");
    Flow* croot = cp + (n - 1);
    if (n_unique == n) {  // nothing collapsed: the copies' graph is the canonical one
        if (lowered) *lowered = std::move(ev);
        return croot;
    }
    // deps re-pointed at each class's first copy (equal digests by
    // construction, so no digest changes)
    parallel_ranges(n, 16384, lower_threads(e), [&](size_t, size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            for (Flow*& d : cp[i].Deps) d = cp + first[d - cp];
            if (cp[i].MapFlow) cp[i].MapFlow = cp + first[cp[i].MapFlow - cp];
        }
    });
    pc.lap("canonicalize: deps re-pointed");
    if (lowered) {
        // the copies' lowered jobs, collapsed the same way: handed over
        ev->collapse(first);
        *lowered = std::move(ev);
    }
    return cp + first[n - 1];
}

// Canonicalize's collapse (flowMap.Put: the first copy with a digest wins,
// flow.go:826-839) applied to the copies' lowered jobs (block 0, copy i in
// slot slot0 + i): a duplicate's logical and physical jobs are dropped,
// every hole naming a duplicate's slot names its class's first copy (equal
// digests, so no digest changes), and a duplicate's lookups alias its first
// copy.  The compacted table (templates left in place in the blob) is loaded
// and takes the copies' graph's slot table as it stands (rf_graph_adopt_slots:
// every kept job is one of the copies' jobs, reading slots of equal digests),
// so nothing is lowered again and nothing is recomputed.
void Eval::collapse(const std::vector<uint32_t>& first) {
    PhaseClock pc;
    Block& b = blocks_.front();
    const uint32_t s0 = b.slot0, nb = (uint32_t)b.n;
    if (first.size() != b.n) throw Error(RF_EINVAL, "collapse: class table size");
    std::vector<uint8_t> drop(n_slots_, 0);
    size_t dups = 0;
    for (uint32_t i = 0; i < nb; ++i)
        if (first[i] != i) {
            if (first[i] > i) throw Error(RF_EINVAL, "collapse: a class's first copy follows a member");
            ++dups;
            drop[s0 + i] = 1;
            if (b.phys[i] != ~0u) drop[b.phys[i]] = 1;
        }
    const size_t J = out_slot_.size();
    constexpr size_t kGrain = 1 << 16;
    const size_t nr = (J + kGrain - 1) / kGrain;
    std::vector<uint64_t> kj(nr + 1, 0), kh(nr + 1, 0);  // kept jobs / holes before each range
    const unsigned th = lower_threads(e_);
    parallel_ranges(J, kGrain, th, [&](size_t r, size_t lo, size_t hi) {
        uint64_t j = 0, h = 0;
        for (size_t k = lo; k < hi; ++k)
            if (!drop[out_slot_[k]]) {
                ++j;
                h += hole_ptr_[k + 1] - hole_ptr_[k];
            }
        kj[r + 1] = j;
        kh[r + 1] = h;
    });
    for (size_t r = 0; r < nr; ++r) {
        kj[r + 1] += kj[r];
        kh[r + 1] += kh[r];
    }
    detail::RawVec<uint32_t> out(kj[nr]), tlen(kj[nr]), hpos(kh[nr]), hslot(kh[nr]);
    detail::RawVec<uint64_t> toff(kj[nr]), hptr(kj[nr] + 1);
    hptr[0] = 0;
    parallel_ranges(J, kGrain, th, [&](size_t r, size_t lo, size_t hi) {
        uint64_t j = kj[r], h = kh[r];
        for (size_t k = lo; k < hi; ++k) {
            if (drop[out_slot_[k]]) continue;
            out[j] = out_slot_[k];
            tlen[j] = tmpl_len_[k];
            toff[j] = tmpl_off_[k];
            for (uint64_t x = hole_ptr_[k]; x < hole_ptr_[k + 1]; ++x, ++h) {
                uint32_t s = hole_slot_[x];
                if (s - s0 < nb) s = s0 + first[s - s0];
                hpos[h] = hole_pos_[x];
                hslot[h] = s;
            }
            hptr[++j] = h;
        }
    });
    out_slot_.swap(out);
    tmpl_len_.swap(tlen);
    tmpl_off_.swap(toff);
    hole_ptr_.swap(hptr);
    hole_pos_.swap(hpos);
    hole_slot_.swap(hslot);
    b.canon = first;
    collapsed_ = dups;
    pc.lap("canonicalize: collapse (threads)");
    rf_graph* copies = g_;
    g_ = nullptr;
    try {
        load();
        Check(rf_graph_adopt_slots(g_, copies));
    } catch (...) {
        rf_graph_destroy(copies);
        throw;
    }
    rf_graph_destroy(copies);
    pc.lap("canonicalize: collapsed load + slot table adopted");
}

// ---- Liveset ---------------------------------------------------------------------
Liveset::Liveset(Engine& e, uint64_t m, uint64_t k) { Check(rf_bloom_new(e.ctx(), m, k, &b_)); }

Liveset Liveset::FromJSON(Engine& e, const std::string& js) {
    rf_bloom* b = nullptr;
    Check(rf_bloom_load_json(e.ctx(), js.data(), js.size(), &b));
    return Liveset(b);
}

Liveset::~Liveset() {
    if (b_) rf_bloom_destroy(b_);
}

void Liveset::Add(const std::vector<Digest>& ds) {
    if (!ds.empty()) Check(rf_bloom_add(b_, ds[0].b.data(), ds.size()));
}

std::vector<bool> Liveset::Contains(const std::vector<Digest>& ds) {
    std::vector<uint8_t> out(ds.size());
    if (!ds.empty()) Check(rf_bloom_probe(b_, ds[0].b.data(), ds.size(), out.data()));
    return std::vector<bool>(out.begin(), out.end());
}

std::string Liveset::MarshalJSON() const {
    uint64_t n = 0;
    rf_bloom_marshal_json(b_, nullptr, 0, &n);
    std::string out(n, '\0');
    Check(rf_bloom_marshal_json(b_, reinterpret_cast<uint8_t*>(out.data()), n, &n));
    return out;
}

std::pair<std::vector<uint64_t>, int64_t> Liveset::Collect(const std::vector<Digest>& objs,
                                                           const std::vector<int64_t>& sizes) {
    std::vector<uint64_t> dead(objs.size() + 1);
    uint64_t nd = 0;
    int64_t bytes = 0;
    if (!objs.empty())
        Check(rf_bloom_collect(b_, objs[0].b.data(), sizes.empty() ? nullptr : sizes.data(), objs.size(),
                               dead.data(), &nd, &bytes));
    dead.resize(nd);
    return {dead, bytes};
}

// ---- assoc -------------------------------------------------------------------
Assoc::Assoc(Engine& e, uint64_t capacity) { Check(rf_assoc_new(e.ctx(), capacity, &a_)); }
Assoc::~Assoc() {
    if (a_) rf_assoc_destroy(a_);
}

std::vector<int> Assoc::PutBatch(AssocKind kind, const std::vector<Digest>& expect, const std::vector<Digest>& keys,
                                 const std::vector<Digest>& vals) {
    if (keys.size() != vals.size() || (!expect.empty() && expect.size() != keys.size()))
        throw Error(RF_EINVAL, "assoc put: mismatched batch sizes");
    std::vector<int32_t> st(keys.size());
    if (!keys.empty())
        Check(rf_assoc_put(a_, kind, expect.empty() ? nullptr : expect[0].b.data(), keys[0].b.data(),
                           vals[0].b.data(), keys.size(), st.data()));
    return std::vector<int>(st.begin(), st.end());
}

void Assoc::Put(AssocKind kind, const Digest& expect, const Digest& k, const Digest& v) {
    const int st = PutBatch(kind, {expect}, {k}, {v})[0];
    if (st == RF_EPRECONDITION)  // testutil/assoc.go:38-40: errors.Precondition
        throw Error(RF_EPRECONDITION, "expected value " + expect.String() + ", have a different value");
}

std::vector<std::pair<int, Digest>> Assoc::Lookup(AssocKind kind, const std::vector<std::vector<Digest>>& node_keys,
                                                  int repair, const FsidCheck& usable, const FsidCheck& verified) {
    if (repair < 0 || repair > 2) throw Error(RF_EINVAL, "repair must be 0, 1 or 2");
    std::vector<uint64_t> ptr{0};
    std::vector<uint8_t> flat;
    for (const auto& ks : node_keys) {
        for (const Digest& k : ks) flat.insert(flat.end(), k.b.begin(), k.b.end());
        ptr.push_back(ptr.back() + ks.size());
    }
    const size_t n = node_keys.size(), nk = ptr.back();
    std::vector<std::pair<int, Digest>> out(n, {-1, Digest{}});
    if (!n) return out;
    std::vector<int32_t> which(n);
    std::vector<uint8_t> vals(32 * n), found(nk + 1), kvals(32 * nk + 32);
    Check(rf_assoc_lookup(a_, (int)kind, flat.empty() ? nullptr : flat.data(), ptr.data(), n, which.data(),
                          vals.data(), found.data(), kvals.data()));
    // per node: the first found key whose fsid the caller can use
    std::vector<int32_t> rep(n, -1);
    std::vector<uint8_t> rvals(32 * n, 0);
    for (size_t i = 0; i < n; ++i) {
        for (uint64_t k = ptr[i]; k < ptr[i + 1]; ++k) {
            if (!found[k]) continue;
            Digest v;
            memcpy(v.b.data(), kvals.data() + 32 * k, 32);
            if (usable && !usable(i, v)) continue;
            out[i] = {(int)(k - ptr[i]), v};
            break;
        }
        if (out[i].first >= 0 && (!verified || verified(i, out[i].second))) {
            rep[i] = out[i].first;
            memcpy(rvals.data() + 32 * i, out[i].second.b.data(), 32);
        }
    }
    if (repair)
        Check(rf_assoc_repair(a_, (int)kind, flat.empty() ? nullptr : flat.data(), ptr.data(), n, rep.data(),
                              rvals.data(), repair == 2 ? found.data() : nullptr));
    return out;
}

std::vector<std::optional<Digest>> Assoc::GetBatch(AssocKind kind, const std::vector<Digest>& keys) {
    std::vector<Digest> vals(keys.size());
    std::vector<uint8_t> found(keys.size());
    if (!keys.empty())
        Check(rf_assoc_get(a_, kind, keys[0].b.data(), keys.size(), vals[0].b.data(), found.data()));
    std::vector<std::optional<Digest>> out(keys.size());
    for (size_t i = 0; i < keys.size(); ++i)
        if (found[i]) out[i] = vals[i];
    return out;
}

std::pair<Digest, Digest> Assoc::Get(AssocKind kind, const Digest& k) {
    auto v = GetBatch(kind, {k})[0];
    if (!v) throw Error(RF_ENOTFOUND, "key does not exist");  // testutil/assoc.go:51-54
    return {k, *v};
}

std::pair<Digest, Digest> Assoc::GetAbbrev(AssocKind kind, const std::string& hex) {
    if (hex.size() < 8 || hex.size() > 64) throw Error(RF_EINVAL, "abbreviated key needs 8..64 hex digits");
    Digest q;
    for (size_t i = 0; i < hex.size(); ++i) {
        const char c = hex[i];
        const int v = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
        if (v < 0) throw Error(RF_EINVAL, "bad hex digit in abbreviated key");
        q.b[i / 2] |= (uint8_t)(i % 2 ? v : v << 4);
    }
    const uint8_t nh = (uint8_t)hex.size();
    Digest ko, vo;
    int32_t st = 0;
    Check(rf_assoc_get_abbrev(a_, kind, q.b.data(), &nh, 1, ko.b.data(), vo.b.data(), &st));
    if (st == RF_ENOTFOUND) throw Error(RF_ENOTFOUND, "lookup " + hex + ": key does not exist");
    if (st == RF_EINVAL) throw Error(RF_EINVAL, "lookup " + hex + ": more than one key matched");
    return {ko, vo};
}

void Delete(Assoc& a, AssocKind kind, const Digest& k) { a.Put(kind, Digest{}, k, Digest{}); }

}  // namespace reflow

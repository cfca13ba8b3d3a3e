// reflow_host.hpp -- C++ host-side mirror of Reflow's memoization API over the
// C-ABI in reflow_hip.h.
//
// The reference is Go (no Go toolchain in this image), so the host side above
// the ABI is C++ with the reference's names and meaning:
//   Digest / WriteDigest      grailbio/base/digest (00 05 || sha256)
//   Digester                  reflow.Digester (flow.go:36), batched on the GPU
//   File / Fileset            executor.go:25-38, WriteDigest :214-233
//   Install                   Executor.install (local/executor.go:514-557)
//   Op / Config / Flow        flow.go:40-301, Op.DigestString op_string.go:15-21
//   flow::Exec/Intern/...     test/flow/constructor.go:17-74
//   Eval                      Flow.Digest / PhysicalDigest / CacheKeys /
//                             Canonicalize (flow.go:653-843), lowered to
//                             rf_graph jobs and computed by the HIP kernels
//   Liveset                   bloomlive.T (internal/bloomlive/bloomlive.go),
//                             MarshalJSON, Repository.Collect
//   Assoc                     assoc.Assoc (assoc/assoc.go) on the HBM table
//   MarshalJSON               json.Marshal(Fileset), the CacheWrite value
// Every digest is computed by libreflow_hip.so on the device.
#pragma once

#include <array>
#include <cstring>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <new>
#include <optional>
#include <string>
#include <unordered_map>
#include <vector>

#include "reflow_hip.h"

namespace reflow {

struct Error : std::exception {
    int code;
    std::string msg;
    Error(int c, std::string m) : code(c), msg(std::move(m)) {}
    const char* what() const noexcept override { return msg.c_str(); }
};

// ---- digest ----------------------------------------------------------------
struct Digest {
    std::array<uint8_t, 32> b{};
    bool IsZero() const;
    std::string Hex() const;
    std::string String() const;  // "sha256:<64 hex>"
    std::string Short() const;   // "sha256:<8 hex>"
    bool Less(const Digest& o) const { return b < o.b; }
    bool operator==(const Digest& o) const { return b == o.b; }
    bool operator!=(const Digest& o) const { return b != o.b; }
    static bool Parse(const std::string& s, Digest* out);
};
struct DigestHash {
    size_t operator()(const Digest& d) const {
        uint64_t w[4];
        memcpy(w, d.b.data(), sizeof w);
        uint64_t h = (w[0] ^ (w[1] << 17 | w[1] >> 47) ^ (w[2] << 31 | w[2] >> 33) ^ (w[3] << 47 | w[3] >> 17));
        h ^= h >> 32;
        h *= 0x9E3779B97F4A7C15ull;
        return (size_t)(h ^ (h >> 29));
    }
};
// digest.WriteDigest: big-endian uint16(crypto.SHA256 = 5) then the 32 bytes.
void WriteDigest(std::string& w, const Digest& d);

namespace detail {
// Allocator for tables that are probed at random (the lowering's maps hold
// tens of millions of entries, hundreds of MB): from 4 MB on, 2 MB-aligned
// and marked for transparent huge pages, so a probe costs a cache miss but
// rarely a TLB miss as well.  Falls back to plain pages where the kernel
// declines.
void* huge_page_alloc(size_t bytes);
void huge_page_free(void* p, size_t bytes) noexcept;
template <class T>
struct HugePageAlloc {
    using value_type = T;
    HugePageAlloc() = default;
    template <class U>
    HugePageAlloc(const HugePageAlloc<U>&) noexcept {}
    T* allocate(size_t n) { return static_cast<T*>(huge_page_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t n) noexcept { huge_page_free(p, n * sizeof(T)); }
    template <class U>
    bool operator==(const HugePageAlloc<U>&) const noexcept { return true; }
    template <class U>
    bool operator!=(const HugePageAlloc<U>&) const noexcept { return false; }
};
// Open-addressing hash map (linear probing, backward-shift erase) for the
// lowering's hot lookups -- Flow pointers and File IDs, tens of millions of
// them per Eval: one probe run per lookup instead of a node-based map's
// allocation and pointer chase.
template <class K, class V, class Hash, class Eq = std::equal_to<K>>
class FlatMap {
   public:
    size_t size() const { return n_; }
    void reserve(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n) cap <<= 1;
        if (cap > slots_.size()) rehash(cap);
    }
    V* find(const K& k) {
        if (slots_.empty()) return nullptr;
        for (size_t i = Hash{}(k) & mask_;; i = (i + 1) & mask_) {
            Slot& s = slots_[i];
            if (!s.used) return nullptr;
            if (Eq{}(s.k, k)) return &s.v;
        }
    }
    const V* find(const K& k) const { return const_cast<FlatMap*>(this)->find(k); }
    // a hint that k is about to be looked up: its probe run's first slot
    // into the cache (a lookup into a table of hundreds of MB is a miss)
    void prefetch(const K& k) const {
        if (!slots_.empty()) __builtin_prefetch(&slots_[Hash{}(k) & mask_]);
    }
    // k must be absent
    V& insert(const K& k, V v) {
        if (2 * (n_ + 1) > slots_.size()) rehash(slots_.empty() ? 16 : 2 * slots_.size());
        size_t i = Hash{}(k) & mask_;
        while (slots_[i].used) i = (i + 1) & mask_;
        slots_[i] = Slot{k, std::move(v), true};
        ++n_;
        return slots_[i].v;
    }
    bool erase(const K& k) {
        if (slots_.empty()) return false;
        size_t i = Hash{}(k) & mask_;
        for (;; i = (i + 1) & mask_) {
            if (!slots_[i].used) return false;
            if (Eq{}(slots_[i].k, k)) break;
        }
        // backward shift: move later members of the run into the hole
        for (size_t j = (i + 1) & mask_;; j = (j + 1) & mask_) {
            if (!slots_[j].used) break;
            const size_t h = Hash{}(slots_[j].k) & mask_;
            if (((j - h) & mask_) >= ((j - i) & mask_)) {
                slots_[i] = std::move(slots_[j]);
                i = j;
            }
        }
        slots_[i].used = false;
        --n_;
        return true;
    }
    template <class F>
    void for_each(F f) const {
        for (const Slot& s : slots_)
            if (s.used) f(s.k, s.v);
    }
    template <class F>
    void for_each_mut(F f) {
        for (Slot& s : slots_)
            if (s.used) f(s.k, s.v);
    }

   private:
    struct Slot {
        K k{};
        V v{};
        bool used = false;
    };
    void rehash(size_t cap) {
        std::vector<Slot, HugePageAlloc<Slot>> old(cap);
        old.swap(slots_);
        mask_ = cap - 1;
        n_ = 0;
        for (Slot& s : old)
            if (s.used) insert(s.k, std::move(s.v));
    }
    std::vector<Slot, HugePageAlloc<Slot>> slots_;
    size_t mask_ = 0, n_ = 0;
};
// std::vector whose resize default-initialises (no zero fill of the new
// elements): gigabytes of lowered templates are written once, in parallel
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
template <class T>
using RawVec = std::vector<T, DefaultInitAlloc<T>>;
struct PtrHash {
    size_t operator()(const void* p) const {
        uint64_t x = (uint64_t)(uintptr_t)p;
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 33;
        return (size_t)x;
    }
};
}  // namespace detail

// ---- engine (one rf_ctx per GPU) -------------------------------------------
class Engine {
   public:
    explicit Engine(int device = 0);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    rf_ctx* ctx() const { return ctx_; }

   private:
    rf_ctx* ctx_ = nullptr;
};

void Check(int rc);  // throws Error with rf_last_error()

// reflow.Digester: FromBytes/FromString, batched.
class Digester {
   public:
    explicit Digester(Engine& e) : e_(e) {}
    Digest FromBytes(const std::string& b) { return FromBytesBatch({b})[0]; }
    Digest FromString(const std::string& s) { return FromBytes(s); }
    std::vector<Digest> FromBytesBatch(const std::vector<std::string>& msgs);

   private:
    Engine& e_;
};

// ---- values ------------------------------------------------------------------
struct File {
    Digest ID;
    int64_t Size = 0;
};

struct Fileset {
    std::optional<std::vector<Fileset>> List;  // non-nil List wins (executor.go:216-219)
    std::map<std::string, File> Map;           // std::map = sort.Strings order
    void WriteDigest(std::string& w) const;
    size_t N() const;
    bool Empty() const;
};

// Fileset.Digest for many filesets in one device call.
std::vector<Digest> FilesetDigests(Engine& e, const std::vector<const Fileset*>& v);
// json.Marshal(Fileset) (eval.go:1961-1967; host code) and the value digests
// CacheWrite stores under each cache key (SHA-256 on the GPU).
std::string MarshalJSON(const Fileset& v);
std::vector<Digest> FilesetValueDigests(Engine& e, const std::vector<const Fileset*>& v);
// Executor.install (local/executor.go:514-557): walk `path` like
// internal/walker (symlinks followed, missing paths skipped, sorted
// depth-first), digest every file on the GPU -> Fileset{Map: relpath -> File}.
// *digest (optional) receives the Fileset's digest computed alongside.
Fileset Install(Engine& e, const std::string& path, Digest* digest = nullptr);

// ---- flows -------------------------------------------------------------------
enum Op : int {
    OpExec = 1, OpIntern, OpExtern, OpGroupby, OpMap, OpCollect, OpMerge, OpVal, OpPullup, OpK,
    OpCoerce, OpRequirements, OpData
};
// op_string.go:15-21 (the generated table is one entry stale: OpData -> "maxOp")
std::string DigestString(Op op);

struct ExecArg {
    bool Out = false;
    int Index = 0;
};

struct Config {
    bool HashV1 = false;
    void Merge(const Config& d) { HashV1 = HashV1 || d.HashV1; }
};

// A Flow's Fileset value, read like std::optional<Fileset> but SHARED by a
// node and its copies: Go's Flow.Copy (flow.go:818-843) copies the struct,
// and a Fileset's Map is a reference there, so the copies Canonicalize makes
// share their originals' values instead of duplicating every map (on a
// 10M-node graph the value copies were most of the copy phase).  Assigning a
// Fileset gives the node a value of its own; writing through * or -> is seen
// by every node sharing it, as in Go.
class FlowValue {
   public:
    FlowValue() = default;
    FlowValue(std::nullopt_t) {}
    FlowValue(const Fileset& v) : p_(std::make_shared<Fileset>(v)) {}
    FlowValue(Fileset&& v) : p_(std::make_shared<Fileset>(std::move(v))) {}
    FlowValue(const std::optional<Fileset>& v) {
        if (v) p_ = std::make_shared<Fileset>(*v);
    }
    FlowValue& operator=(std::nullopt_t) {
        p_.reset();
        return *this;
    }
    FlowValue& operator=(const Fileset& v) {
        p_ = std::make_shared<Fileset>(v);
        return *this;
    }
    FlowValue& operator=(Fileset&& v) {
        p_ = std::make_shared<Fileset>(std::move(v));
        return *this;
    }
    explicit operator bool() const { return p_ != nullptr; }
    bool has_value() const { return p_ != nullptr; }
    const Fileset& operator*() const { return *p_; }
    Fileset& operator*() { return *p_; }
    const Fileset* operator->() const { return p_.get(); }
    Fileset* operator->() { return p_.get(); }
    const Fileset& value() const {
        if (!p_) throw std::bad_optional_access();
        return *p_;
    }
    void reset() { p_.reset(); }

   private:
    std::shared_ptr<Fileset> p_;
};

struct Flow {
    Op op = OpVal;
    Flow* Parent = nullptr;
    std::vector<Flow*> Deps;
    Config config;
    std::string Image, Cmd;           // OpExec
    std::string URL;                  // OpIntern/OpExtern: url.URL.String() bytes
    std::string Re, Repl;             // OpGroupby/OpCollect: regexp.String(), Repl
    Flow* MapFlow = nullptr;          // OpMap (MapInit already applied)
    std::optional<std::vector<ExecArg>> Argmap;
    Digest FlowDigest;                // OpVal (non-Fileset), OpK, OpCoerce
    bool Done = false;                // State == FlowDone
    FlowValue Value;                  // Fileset value (shared with copies)
    bool Err = false;                 // error values digest randomly (not supported here)
    std::string Data;                 // OpData
};

namespace detail {
using PtrIndex = FlatMap<const Flow*, uint32_t, PtrHash>;
// Canonicalize's walk (flow.go:820-839, the order of flowMap.Put): the nodes
// reachable from root through Deps and MapFlow in post-order (deps, then the
// map flow, then the node) into post, each one's position into index.  A
// wide root's children are walked in groups on up to `threads` host threads;
// the order is the sequential walk's exactly.
void PostOrder(Flow* root, unsigned threads, std::vector<Flow*>& post, PtrIndex& index);
}  // namespace detail

// Owns Flow nodes (the Go GC's job in the reference).
class FlowArena {
   public:
    Flow* New(Flow f) {
        nodes_.push_back(std::move(f));
        return &nodes_.back();
    }
    // n default-constructed nodes, contiguous (an Eval then maps a node of
    // the block to its slot by address, no hash lookup)
    Flow* NewN(size_t n) {
        return NewN(n, [](Flow* f, size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; ++i) new (f + i) Flow();
        });
    }
    // n contiguous nodes, each constructed by make(block, lo, hi) -- placement
    // new of [lo, hi) -- which may split the range over threads (Canonicalize
    // copy-constructs its copies in place: no default construction first,
    // and the pages are first touched by the threads that fill them; a
    // multi-GB block sits on huge-page-advised storage, so filling it is not
    // a page fault per 4 KiB).  make must construct every node, or throw
    // having constructed none.
    template <class Make>
    Flow* NewN(size_t n, Make make) {
        Block b;
        b.n = n ? n : 1;
        b.p = static_cast<Flow*>(detail::huge_page_alloc(b.n * sizeof(Flow)));
        try {
            make(b.p, size_t(0), n);
            if (!n) new (b.p) Flow();
        } catch (...) {
            detail::huge_page_free(b.p, b.n * sizeof(Flow));
            throw;
        }
        blocks_.push_back(b);
        return b.p;
    }
    FlowArena() = default;
    FlowArena(const FlowArena&) = delete;
    FlowArena& operator=(const FlowArena&) = delete;
    ~FlowArena() {
        for (Block& b : blocks_) {
            for (size_t i = 0; i < b.n; ++i) b.p[i].~Flow();
            detail::huge_page_free(b.p, b.n * sizeof(Flow));
        }
    }

   private:
    struct Block {
        Flow* p = nullptr;
        size_t n = 0;
    };
    std::deque<Flow> nodes_;
    std::vector<Block> blocks_;
};

// test/flow/constructor.go:17-74
namespace flow {
Flow* Exec(FlowArena& a, const std::string& image, const std::string& cmd, std::vector<Flow*> deps);
Flow* Intern(FlowArena& a, const std::string& url);
Flow* Extern(FlowArena& a, const std::string& url, Flow* dep);
Flow* Groupby(FlowArena& a, const std::string& re, Flow* dep);
Flow* Collect(FlowArena& a, const std::string& re, const std::string& repl, Flow* dep);
// MapFunc is applied to &Flow{Op: OpVal, Value: Fileset{}} (MapInit, flow.go:315-317)
template <class F>
Flow* Map(FlowArena& a, F fn, Flow* dep) {
    Flow* v = a.New(Flow{});
    v->op = OpVal;
    v->Value = Fileset{};
    Flow f;
    f.op = OpMap;
    f.Deps = {dep};
    f.MapFlow = fn(v);
    return a.New(std::move(f));
}
Flow* Merge(FlowArena& a, std::vector<Flow*> deps);
Flow* Pullup(FlowArena& a, std::vector<Flow*> deps);
Flow* Val(FlowArena& a, const Fileset& v);
Flow* Data(FlowArena& a, const std::string& b);
}  // namespace flow

class Eval;
// Canonicalize (flow.go:814-843): copies merged with `config`, semantically
// equal nodes (equal digests) collapsed to the first one in visit order.
// The copies' digests come from the device: an Eval (file slots on) over the
// copies, lowered, loaded and fully recomputed.  `lowered` (optional): that
// Eval handed over ready for FlowDigest / CacheKeys / SetFileID + Recompute
// of the canonical graph -- the caller's Eval.Add + Build of the same graph
// (what a fresh Eval does after Canonicalize, eval.go:240-272) is skipped.
// When copies collapsed, the handed-over Eval's duplicate jobs are dropped,
// holes that named a duplicate name its class's first copy, and a duplicate's
// lookups answer with its first copy's slots (Eval::Collapsed() counts them);
// the table is reloaded and recomputed without a second lowering.
Flow* Canonicalize(Engine& e, FlowArena& arena, Flow* root, Config config,
                   const std::string& universe = "", std::unique_ptr<Eval>* lowered = nullptr);

// Batched Flow.Digest / PhysicalDigest / CacheKeys over a whole DAG: the DAG
// is lowered to rf_graph jobs (one logical job per node, one physical job per
// OpExec/OpExtern whose deps are Done) and evaluated on the device.  With
// file_slots, every File.ID inside Fileset values becomes an input slot, so
// SetFileID + Recompute re-derive only the dependents (incremental).
class Eval {
   public:
    Eval(Engine& e, std::string universe = "", bool file_slots = false);
    ~Eval();
    void Add(Flow* root);
    void Build();  // rf_graph_load + full recompute
    Digest FlowDigest(const Flow* f) const;
    std::optional<Digest> PhysicalDigest(const Flow* f) const;
    std::vector<Digest> CacheKeys(const Flow* f) const;
    // Change one File ID wherever Fileset values reference it (needs file_slots).
    void SetFileID(const Digest& old_id, const Digest& new_id);
    uint64_t Recompute(bool full = false);
    size_t Jobs() const { return out_slot_.size(); }
    size_t Collapsed() const { return collapsed_; }  // copies Canonicalize collapsed into a first copy

   private:
    friend Flow* Canonicalize(Engine&, FlowArena&, Flow*, Config, const std::string&, std::unique_ptr<Eval>*);
    using Holes = std::vector<std::pair<uint32_t, uint32_t>>;  // (byte pos, slot)
    // File IDs referenced from a job's material (file slots): (its hole's
    // index in the job, the ID) -- slots are given after the parallel phase
    using FileRefs = std::vector<std::pair<uint32_t, Digest>>;
    struct Part;  // one range of nodes' jobs, built by one thread (reflow_host.cpp)
    // a contiguous run of nodes (FlowArena::NewN) whose logical slots are
    // slot0 + index: found by address, never hashed
    struct Block {
        const Flow* base;
        size_t n;
        uint32_t slot0;
        std::vector<uint32_t> phys;  // physical slot per node, ~0u: none
        std::vector<uint32_t> canon;  // (after a collapse) node -> its class's first node; empty: itself
        size_t at(const Flow* f) const {
            const size_t i = (size_t)(f - base);
            return canon.empty() ? i : canon[i];
        }
    };
    void material(const Flow* f, std::string& out, Holes& holes, FileRefs& files) const;
    void fileset_material(const Fileset& v, std::string& out, Holes& holes, FileRefs& files) const;
    void lower_nodes(const std::vector<const Flow*>* nodes, const Block* blk, const std::vector<uint32_t>& phys);
    void add_block(const Flow* base, size_t n);
    void collapse(const std::vector<uint32_t>& first);
    void load();
    const uint32_t* slot_of(const Flow* f) const;
    const uint32_t* phys_slot_of(const Flow* f) const;
    uint32_t new_slot() { return n_slots_++; }

    Engine& e_;
    std::string U_;
    bool file_slots_;
    uint32_t n_slots_ = 0;
    size_t collapsed_ = 0;
    // the jobs, as the rf_graph_desc arrays
    // (grown without zero-filling: the parallel append writes every element)
    detail::RawVec<uint32_t> out_slot_, tmpl_len_, hole_pos_, hole_slot_;
    detail::RawVec<uint64_t> tmpl_off_, hole_ptr_{0};
    detail::RawVec<char> blob_;
    std::vector<Block> blocks_;
    detail::FlatMap<const Flow*, uint32_t, detail::PtrHash> logical_, physical_;
    // File ID -> its input slot, in kFileShards shards by hash (the lowering
    // resolves a batch's IDs shard by shard on host threads)
    static constexpr unsigned kFileShards = 64;
    static unsigned file_shard(const Digest& id) { return (unsigned)(DigestHash{}(id) >> 58); }
    std::vector<detail::FlatMap<Digest, uint32_t, DigestHash>> file_slot_{kFileShards};
    size_t n_files() const {
        size_t n = 0;
        for (const auto& m : file_slot_) n += m.size();
        return n;
    }
    rf_graph* g_ = nullptr;
    mutable std::vector<uint8_t> cache_;  // all slots after the last recompute
    mutable bool cache_ok_ = false;
    void fetch() const;
};

// bloomlive.T over the device filter: Contains batched.
class Liveset {
   public:
    Liveset(Engine& e, uint64_t m, uint64_t k);          // bloom.New
    static Liveset FromJSON(Engine& e, const std::string& js);
    Liveset(Liveset&& o) noexcept : b_(o.b_) { o.b_ = nullptr; }
    ~Liveset();
    void Add(const std::vector<Digest>& ds);
    std::vector<bool> Contains(const std::vector<Digest>& ds);
    std::string MarshalJSON() const;  // bloomlive.go:38-41 (the Go wire form)
    // Repository.Collect (repository/file/repository.go:304-327) over a batch
    // of objects: indices (walk order) of the ones not in the liveset, and
    // their total size.
    std::pair<std::vector<uint64_t>, int64_t> Collect(const std::vector<Digest>& objs,
                                                      const std::vector<int64_t>& sizes);

   private:
    explicit Liveset(rf_bloom* b) : b_(b) {}
    rf_bloom* b_ = nullptr;
};

// assoc.Assoc (assoc/assoc.go:26-38) on the HBM table, with the in-memory
// implementation's semantics (test/testutil/assoc.go:34-56).  Single-key
// calls mirror the Go interface (Put errors with RF_EPRECONDITION, Get with
// RF_ENOTFOUND); the batch forms are what a shim coalesces them into.
enum AssocKind : int { AssocFileset = 0 };
class Assoc {
   public:
    explicit Assoc(Engine& e, uint64_t capacity = 1024);
    ~Assoc();
    Assoc(const Assoc&) = delete;
    Assoc& operator=(const Assoc&) = delete;
    void Put(AssocKind kind, const Digest& expect, const Digest& k, const Digest& v);
    // returns (expanded key, value); an abbreviated key is given as its hex prefix
    std::pair<Digest, Digest> Get(AssocKind kind, const Digest& k);
    std::pair<Digest, Digest> GetAbbrev(AssocKind kind, const std::string& hex_prefix);
    std::vector<int> PutBatch(AssocKind kind, const std::vector<Digest>& expect, const std::vector<Digest>& keys,
                              const std::vector<Digest>& vals);
    std::vector<std::optional<Digest>> GetBatch(AssocKind kind, const std::vector<Digest>& keys);
    // Eval.lookup's assoc step for many nodes (eval.go:1172-1258), batched:
    // one Get over every node's cache keys; per node the first key (CacheKeys
    // order) with a value that `usable` accepts -- the caller's unmarshal of
    // the fsid; eval.go:1210-1218 moves on to the next key when it fails --
    // or -1.  Then read repair (0 none, 1 blind as the reference, 2 precise:
    // missing keys only) for the nodes whose value `verified` passes (the
    // missing()/RecomputeEmpty checks of eval.go:1227-1246); null callbacks
    // accept everything.
    using FsidCheck = std::function<bool(size_t node, const Digest& fsid)>;
    std::vector<std::pair<int, Digest>> Lookup(AssocKind kind, const std::vector<std::vector<Digest>>& node_keys,
                                               int repair, const FsidCheck& usable = nullptr,
                                               const FsidCheck& verified = nullptr);

   private:
    rf_assoc* a_ = nullptr;
};
void Delete(Assoc& a, AssocKind kind, const Digest& k);  // assoc.go:40-43

}  // namespace reflow

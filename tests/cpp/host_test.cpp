// host_test.cpp -- the reference's digest tests, restated against the C++ host
// mirror (include/reflow_hip_host.hpp) running on the device.
//   TestDigestStability   flow_test.go:24-44
//   TestCanonicalize      flow_test.go:46-58
//   TestCanonicalizeHandOver  collapsed copies: the handed-over Eval == a fresh lowering
//   TestValueDigest       executor_test.go:62-86
//   TestDigestExec        syntax/digest_test.go:13-29 (the evaluated flow chain)
//   TestCacheKeys         flow.go:764-802 (physical key first)
//   TestIncremental       SetFileID + Recompute == a fresh evaluation
//   TestLiveset           bloomlive Contains over Add, MarshalJSON, Collect
//   TestAssoc             assoc.Assoc: test/testutil/assoc.go semantics, abbreviations
// Exit status 0 iff every check passes.
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <string>

#include "reflow_host.hpp"

using namespace reflow;

static int failures = 0;
#define EXPECT(cond, ...)                                   \
    do {                                                    \
        if (!(cond)) {                                      \
            ++failures;                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                   \
            fprintf(stderr, "\n");                          \
        }                                                   \
    } while (0)

static Flow* stable_flow(FlowArena& a) {
    Flow* intern = flow::Intern(a, "internurl");
    Flow* collect = flow::Collect(a, ".*", "$0", intern);
    Flow* groupby = flow::Groupby(a, "foo-(.*)", collect);
    Flow* mapflow = flow::Map(a, [&](Flow* f) { return flow::Exec(a, "image", "command", {f}); }, groupby);
    return flow::Extern(a, "externurl", mapflow);
}

static void TestDigestStability(Engine& e) {
    const char* v1 = "sha256:5a3a916fe9a11b67f9a0dbd67f6fac0f986dd67803267e79f25f866ca9781e2f";
    const char* v2 = "sha256:02751e46c573a31747a30b05c2b73b2eb556fb45fb4c0aaf88d170f4b5e6d4e7";
    FlowArena a;
    Flow* stable = stable_flow(a);
    Flow* c = Canonicalize(e, a, stable, Config{true});
    Eval ev1(e);
    ev1.Add(c);
    ev1.Build();
    EXPECT(ev1.FlowDigest(c).String() == v1, "V1 got %s", ev1.FlowDigest(c).String().c_str());
    Eval ev2(e);
    ev2.Add(stable);
    ev2.Build();
    EXPECT(ev2.FlowDigest(stable).String() == v2, "V2 got %s", ev2.FlowDigest(stable).String().c_str());
}

static void TestCanonicalize(Engine& e) {
    FlowArena a;
    Flow* i1 = flow::Intern(a, "url");
    Flow* i2 = flow::Intern(a, "url");
    Flow* merged = flow::Merge(a, {i1, i2});
    Eval ev(e);
    ev.Add(merged);
    ev.Build();
    Flow* canon = Canonicalize(e, a, merged, Config{});
    Eval evc(e);
    evc.Add(canon);
    evc.Build();
    EXPECT(evc.FlowDigest(canon) == ev.FlowDigest(merged), "canonical digest changed");
    EXPECT(canon->Deps[0] == canon->Deps[1], "flow is not canonical");
}

static Fileset one(const Digest& id);

// Canonicalize's hand-over when copies collapse: per-branch duplicated
// reference chains (the same Intern -> Exec -> Coerce in every branch) collapse
// to the first branch's; the handed-over Eval drops the duplicates' jobs and
// must equal a fresh lowering of the canonical graph -- digests, cache keys,
// job count, and a SetFileID + Recompute step (count and digests).
static Flow* dup_chains(FlowArena& a, Digester& D, const Digest& ref_id, int branches) {
    std::vector<Flow*> outs;
    for (int b = 0; b < branches; ++b) {
        Flow* r0 = flow::Val(a, one(ref_id));
        Flow* r1 = flow::Exec(a, "bwa", "index %s %s", {r0});
        r1->Argmap = std::vector<ExecArg>{{false, 0}, {true, 0}};
        r1->Done = true;  // (so the mem exec has a physical key, and r1 one of its own)
        r1->Value = one(D.FromString("index"));
        Flow* rd = flow::Val(a, one(D.FromString("reads" + std::to_string(b))));
        Flow* m = flow::Exec(a, "bwa", "mem %s %s %s", {r1, rd});
        m->Argmap = std::vector<ExecArg>{{false, 0}, {false, 1}, {true, 0}};
        outs.push_back(flow::Extern(a, "s3://out/" + std::to_string(b), m));
    }
    return flow::Merge(a, outs);
}

static void TestCanonicalizeHandOver(Engine& e) {
    Digester D(e);
    const Digest ref = D.FromString("reference"), ref2 = D.FromString("reference v2");
    FlowArena a;
    std::unique_ptr<Eval> ev;
    Flow* canon = Canonicalize(e, a, dup_chains(a, D, ref, 5), Config{}, "", &ev);
    EXPECT(ev != nullptr, "no Eval handed over");
    if (!ev) return;
    EXPECT(ev->Collapsed() == 8, "collapsed %zu copies, want 8 (4 branches x Val, Exec)", ev->Collapsed());
    Eval fresh(e, "", true);
    fresh.Add(canon);
    fresh.Build();
    EXPECT(ev->Jobs() == fresh.Jobs(), "handed-over jobs %zu, fresh lowering %zu", ev->Jobs(), fresh.Jobs());
    const Flow* mem = canon->Deps[3]->Deps[0];
    EXPECT(ev->FlowDigest(canon) == fresh.FlowDigest(canon), "root digest");
    EXPECT(ev->CacheKeys(mem).size() == 2 && ev->CacheKeys(mem) == fresh.CacheKeys(mem), "cache keys");
    ev->SetFileID(ref, ref2);
    fresh.SetFileID(ref, ref2);
    const uint64_t n1 = ev->Recompute(), n2 = fresh.Recompute();
    EXPECT(n1 == n2, "incremental counts %llu vs %llu", (unsigned long long)n1, (unsigned long long)n2);
    EXPECT(ev->FlowDigest(canon) == fresh.FlowDigest(canon) && ev->CacheKeys(mem) == fresh.CacheKeys(mem),
           "incremental digests");
    // and against a graph built with the new reference ID from the start
    FlowArena a2;
    Flow* c2 = Canonicalize(e, a2, dup_chains(a2, D, ref2, 5), Config{});
    Eval ev2(e, "", true);
    ev2.Add(c2);
    ev2.Build();
    EXPECT(ev->FlowDigest(canon) == ev2.FlowDigest(c2), "incremental != built with the new ID");
}

static void TestValueDigest(Engine& e) {
    Digester D(e);
    File f1{D.FromString("foo"), 3}, f2{D.FromString("bar"), 3}, f3{D.FromString("a/b/c"), 5};
    Fileset v1, v2, vlist;
    v1.Map = {{"foo", f1}, {"bar", f2}};
    v2.Map = {{"a/b/c", f3}, {"bar", f2}};
    vlist.List = std::vector<Fileset>{v1, v2};
    auto d = FilesetDigests(e, {&v1, &v2, &vlist});
    EXPECT(d[0] != d[1], "did not expect v1, v2 to have the same digest");
    EXPECT(d[2].String() == "sha256:d60e67ce9e89548b502a5ad7968e99caed0d388f0a991b906f41a7ba65adb31f",
           "vlist got %s", d[2].String().c_str());
    EXPECT(vlist.N() == 4, "N");
}

// CacheWrite's assoc value: json.Marshal(Fileset) (eval.go:1961-1967)
static void TestValueJSON(Engine& e) {
    Digester D(e);
    File f1{D.FromString("foo"), 3}, f2{D.FromString("bar"), -1};
    Fileset v1, vlist;
    v1.Map = {{"foo", f1}, {"<b>", f2}};
    vlist.List = std::vector<Fileset>{v1, Fileset{}};
    const std::string want1 = "{\"Fileset\":{\"\\u003cb\\u003e\":{\"ID\":\"" + f2.ID.String() +
                              "\",\"Size\":-1},\"foo\":{\"ID\":\"" + f1.ID.String() + "\",\"Size\":3}}}";
    EXPECT(MarshalJSON(v1) == want1, "json got %s", MarshalJSON(v1).c_str());
    EXPECT(MarshalJSON(vlist) == "{\"List\":[" + want1 + ",{}]}", "list json got %s",
           MarshalJSON(vlist).c_str());
    EXPECT(MarshalJSON(Fileset{}) == "{}", "empty");
    auto d = FilesetValueDigests(e, {&v1, &vlist});
    EXPECT(d[0] == D.FromBytes(want1), "value digest");
    EXPECT(d[1] == D.FromBytes(MarshalJSON(vlist)), "list value digest");
}

static void TestDigestExec(Engine& e) {
    Digester D(e);
    FlowArena a;
    auto coerce = [&](Flow* dep, const char* fd) {
        Flow f;
        f.op = OpCoerce;
        f.Deps = {dep};
        f.FlowDigest = D.FromString(fd);
        return a.New(std::move(f));
    };
    Flow* intern = flow::Intern(a, "s3://blah");
    Flow* c1 = coerce(intern, "file.fs$file");
    Flow k;
    k.op = OpK;
    k.Deps = {c1};
    k.FlowDigest = D.FromString("grail.com/reflow/syntax.Eval.Force");
    Flow* kf = a.New(std::move(k));
    Flow* c2 = coerce(kf, "grail.com/reflow/syntax.coerceFlowToFileset");
    Flow* ex = flow::Exec(a, "ubuntu", " cp %s %s ", {c2});
    ex->Argmap = std::vector<ExecArg>{{false, 0}, {true, 0}};
    Flow* c3 = coerce(ex, "grail.com/reflow/syntax.Eval.coerceExecOutput");
    Eval ev(e);
    ev.Add(c3);
    ev.Build();
    EXPECT(ev.FlowDigest(c3).String() ==
               "sha256:ceff79828962397af02d8e2ea30cf6388f2858e0deefbecaa73fad1c6fc88816",
           "exec chain got %s", ev.FlowDigest(c3).String().c_str());
}

static Fileset one(const Digest& id) {
    Fileset v;
    v.Map = {{".", File{id, 1}}};
    return v;
}

static void TestCacheKeysAndIncremental(Engine& e) {
    Digester D(e);
    FlowArena a;
    Digest ida = D.FromString("a"), idb = D.FromString("b");
    Flow* va = flow::Val(a, one(ida));
    Flow* vb = flow::Val(a, one(idb));
    Flow* ex = flow::Exec(a, "img", "cmd %s %s", {va, vb});
    ex->Argmap = std::vector<ExecArg>{{false, 0}, {false, 1}, {true, 0}};
    Flow* root = flow::Extern(a, "s3://out", ex);
    Eval ev(e, "", /*file_slots=*/true);
    ev.Add(root);
    ev.Build();
    auto keys = ev.CacheKeys(ex);
    EXPECT(keys.size() == 2, "exec over done values has physical + logical keys");
    EXPECT(ev.CacheKeys(root).size() == 1, "extern over an unfinished exec has only the logical key");
    // physical material = FM(va) || FM(vb) || image || cmd || argmap
    std::string pm;
    va->Value->WriteDigest(pm);
    vb->Value->WriteDigest(pm);
    pm += "imgcmd %s %s";
    for (int64_t n : {0, 1, 0}) {
        const uint64_t u = (uint64_t)n;
        for (int i = 0; i < 8; ++i) pm.push_back((char)(u >> (8 * i)));
    }
    EXPECT(keys[0] == D.FromBytes(pm), "physical digest");
    // incremental: change b's ID, compare with a fresh evaluation
    Digest idb2 = D.FromString("b2");
    ev.SetFileID(idb, idb2);
    const uint64_t n = ev.Recompute();
    vb->Value = one(idb2);
    Eval fresh(e, "", true);
    fresh.Add(root);
    fresh.Build();
    for (Flow* f : {va, vb, ex, root})
        EXPECT(ev.FlowDigest(f) == fresh.FlowDigest(f), "incremental != fresh");
    EXPECT(ev.CacheKeys(ex)[0] == fresh.CacheKeys(ex)[0], "physical incremental != fresh");
    EXPECT(n == 4, "recomputed %llu jobs, want 4 (vb, ex, ex physical, root)", (unsigned long long)n);
}

static void TestLiveset(Engine& e) {
    Digester D(e);
    std::vector<std::string> in, out;
    for (int i = 0; i < 1000; ++i) in.push_back("live" + std::to_string(i));
    for (int i = 0; i < 1000; ++i) out.push_back("dead" + std::to_string(i));
    auto din = D.FromBytesBatch(in), dout = D.FromBytesBatch(out);
    Liveset live(e, 14378, 10);  // NewWithEstimates(1000, 0.001)
    live.Add(din);
    auto got = live.Contains(din);
    int fp = 0;
    for (bool b : got) EXPECT(b, "false negative");
    for (bool b : live.Contains(dout)) fp += b;
    EXPECT(fp < 20, "false positives %d", fp);
    Liveset back = Liveset::FromJSON(e, live.MarshalJSON());
    EXPECT(back.MarshalJSON() == live.MarshalJSON(), "JSON round trip");
    std::vector<Digest> objs = din;
    objs.insert(objs.end(), dout.begin(), dout.end());
    auto [dead, bytes] = live.Collect(objs, std::vector<int64_t>(objs.size(), 2));
    auto c = live.Contains(objs);
    size_t j = 0;
    for (size_t i = 0; i < objs.size(); ++i)
        if (!c[i]) EXPECT(j < dead.size() && dead[j++] == i, "collect order at %zu", i);
    EXPECT(j == dead.size() && bytes == 2 * (int64_t)dead.size() && dead.size() + fp == dout.size(),
           "collect %zu dead", dead.size());
}

static void TestAssoc(Engine& e) {
    Digester D(e);
    Assoc a(e, 16);
    Digest k1 = D.FromString("k1"), k2 = D.FromString("k2"), v1 = D.FromString("v1"), v2 = D.FromString("v2");
    bool thrown = false;
    try {
        a.Get(AssocFileset, k1);
    } catch (const Error& er) {
        thrown = er.code == RF_ENOTFOUND;
    }
    EXPECT(thrown, "Get of a missing key is NotExist");
    a.Put(AssocFileset, Digest{}, k1, v1);
    EXPECT(a.Get(AssocFileset, k1).second == v1, "Get after Put");
    thrown = false;
    try {
        a.Put(AssocFileset, v2, k1, v2);  // expect mismatch
    } catch (const Error& er) {
        thrown = er.code == RF_EPRECONDITION;
    }
    EXPECT(thrown && a.Get(AssocFileset, k1).second == v1, "CAS with a wrong expect is Precondition");
    a.Put(AssocFileset, v1, k1, v2);  // CAS succeeds
    EXPECT(a.Get(AssocFileset, k1).second == v2, "CAS");
    a.Put(AssocFileset, Digest{}, k2, v1);
    EXPECT(a.GetAbbrev(AssocFileset, k2.Hex().substr(0, 12)).first == k2, "abbreviated key expands");
    Delete(a, AssocFileset, k1);
    EXPECT(!a.GetBatch(AssocFileset, {k1})[0], "deleted");
    // a batch that touches one key three times applies in order
    auto st = a.PutBatch(AssocFileset, {Digest{}, v1, v2}, {k1, k1, k1}, {v1, v2, v1});
    EXPECT(st[0] == RF_OK && st[1] == RF_OK && st[2] == RF_OK && a.Get(AssocFileset, k1).second == v1,
           "batch order");
    // Eval.lookup (eval.go:1202-1258): physical key absent, logical present ->
    // which = 1; precise read repair fills the physical key
    Digester dg(e);
    const Digest phys = dg.FromString("physical"), logi = dg.FromString("logical");
    a.Put(AssocFileset, Digest{}, logi, v2);
    auto lk = a.Lookup(AssocFileset, {{phys, logi}, {}}, 2);
    EXPECT(lk[0].first == 1 && lk[0].second == v2 && lk[1].first == -1, "lookup first hit");
    EXPECT(a.Get(AssocFileset, phys).second == v2, "precise read repair");
    // a node whose files are missing (verified = false) is not repaired
    const Digest other = dg.FromString("other key");
    lk = a.Lookup(AssocFileset, {{other, logi}}, 1, nullptr, [](size_t, const Digest&) { return false; });
    EXPECT(lk[0].first == 1 && !a.GetBatch(AssocFileset, {other})[0], "no repair of an unverified node");
}

// Executor.install (local/executor.go:514-557): the executor_test.go:86-88
// single-file result, and a small tree whose Fileset digest must equal
// FilesetDigests over the returned Map.
static void TestInstall(Engine& e) {
    char tmpl[] = "/tmp/rf_install_XXXXXX";
    const std::string d = mkdtemp(tmpl);
    auto put = [](const std::string& p, const std::string& b) {
        FILE* f = fopen(p.c_str(), "wb");
        if (f) {
            fwrite(b.data(), 1, b.size(), f);
            fclose(f);
        }
    };
    put(d + "/out", "foobar\n");
    Digester dg(e);
    Fileset one_file = Install(e, d + "/out");
    EXPECT(one_file.Map.size() == 1 && one_file.Map.count(".") &&
               one_file.Map["."].ID == dg.FromString("foobar\n") && one_file.Map["."].Size == 7,
           "install single file -> \".\"");
    mkdir((d + "/t").c_str(), 0755);
    mkdir((d + "/t/a").c_str(), 0755);
    put(d + "/t/a/b", "ab");
    put(d + "/t/a-b", std::string(70000, 'x'));
    put(d + "/t/z", "");
    Digest fsd;
    Fileset t = Install(e, d + "/t", &fsd);
    EXPECT(t.Map.size() == 3 && t.Map["a-b"].Size == 70000 && t.Map["a/b"].ID == dg.FromString("ab"),
           "install tree entries");
    EXPECT(fsd == FilesetDigests(e, {&t})[0], "install fileset digest");
    unlink((d + "/t/a/b").c_str());
    unlink((d + "/t/a-b").c_str());
    unlink((d + "/t/z").c_str());
    rmdir((d + "/t/a").c_str());
    rmdir((d + "/t").c_str());
    unlink((d + "/out").c_str());
    rmdir(d.c_str());
}

int main() {
    try {
        Engine e(0);
        TestDigestStability(e);
        TestCanonicalize(e);
        TestCanonicalizeHandOver(e);
        TestValueDigest(e);
        TestValueJSON(e);
        TestDigestExec(e);
        TestCacheKeysAndIncremental(e);
        TestLiveset(e);
        TestAssoc(e);
        TestInstall(e);
    } catch (const std::exception& ex) {
        fprintf(stderr, "exception: %s\n", ex.what());
        return 2;
    }
    if (failures) {
        fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    printf("PASS\n");
    return 0;
}

// Multi-stream replay of a captured hipGraph (the training step) from a native launch list.
//
// Why: the whole SimCLR step (augment → forward → NT-Xent → backward → LARS, ~500 kernels) can
// be captured into one hipGraph, but the HIP graph executor runs it with less concurrency than
// the eager schedule (the weight gradients on their side stream no longer overlap the
// dgrad/BatchNorm chain: profiles/r4_optimization_log.md), while eager issue costs ~30 µs of
// Python + dispatcher time per kernel.  This executor keeps the captured graph (its node
// parameters: kernel arguments, grids, memset descriptors) but issues it itself:
//
//   * nodes in a topological order that follows capture order (ties by creation index);
//   * each node on one of at most `max_streams` HIP streams: a node continues its parent's
//     stream when it is that parent's heir (the child with the longest path to the end of the
//     graph), else takes a stream whose last node is an ancestor (but not a parent whose heir is
//     still to come), else opens a new stream, else (all streams busy with concurrent work) the
//     stream
//     whose tail was issued earliest;
//   * a cross-stream edge becomes hipEventRecord / hipStreamWaitEvent, pruned with per-stream
//     vector clocks (a wait is issued only when the consumer's stream does not already follow
//     the producer's event transitively);
//   * stream 0 is the caller's current stream; the others fork from it at the start of a replay
//     and join into it at the end, so a replay is stream-ordered like hipGraphLaunch.
//
// gexec_reschedule then re-plans order and streams from measured node durations (list
// scheduling, see there); the replay path is the same.
//
// Host cost per kernel is one hipLaunchKernel with the node's own argument block.  The graph
// must outlive the executor (torch.cuda.CUDAGraph(keep_graph=True) keeps it).
#include <ATen/hip/HIPContext.h>
#include <c10/util/Exception.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <queue>
#include <unordered_map>
#include <vector>

namespace {

#define GX_CHECK(expr)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    TORCH_CHECK(e_ == hipSuccess, "graphexec: ", #expr, " failed: ", hipGetErrorString(e_)); \
  } while (0)

// kSub: any other node (memcpy nodes — HIP does not expose the parameters of one captured from a
// 1-D hipMemcpyAsync —, child graphs, ...) replayed as a one-node executable graph cut from a
// clone of the captured graph
enum NodeKind : int { kKernel = 0, kSub, kMemset, kHost, kEmpty, kEvRecord, kEvWait };

struct Node {
  NodeKind kind = kEmpty;
  hipKernelNodeParams kp{};
  hipGraphExec_t sub = nullptr;
  hipMemsetParams mp{};
  hipHostNodeParams hp{};
  hipEvent_t ext_event = nullptr;
  int stream = 0;
  std::vector<int> waits;  // indices (into `order`) of producer nodes whose event to wait on
  int event = -1;          // index into events if a consumer on another stream waits on it
};

struct Exec {
  std::vector<Node> nodes;  // issue order
  std::vector<std::vector<int>> par;  // parents of every node (positions in `nodes`)
  std::vector<hipStream_t> streams;  // [0] is a placeholder: the caller's stream at replay
  std::vector<hipEvent_t> events;
  hipEvent_t fork = nullptr;
  std::vector<hipEvent_t> joins;
  int nstreams = 1;
  int64_t counts[8] = {0};  // per NodeKind (kKernel..kEvWait) and the number of waits
  ~Exec() {
    for (auto& nd : nodes)
      if (nd.sub) (void)hipGraphExecDestroy(nd.sub);
    for (auto e : events) (void)hipEventDestroy(e);
    for (auto e : joins) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
    for (size_t i = 1; i < streams.size(); ++i) (void)hipStreamDestroy(streams[i]);
  }
};

Exec* as_exec(int64_t h) {
  TORCH_CHECK(h != 0, "graphexec: null handle");
  return reinterpret_cast<Exec*>(h);
}

// a one-node executable graph performing `node` of `g` (cloned, every other node removed)
hipGraphExec_t single_node_exec(hipGraph_t g, hipGraphNode_t node) {
  hipGraph_t c;
  GX_CHECK(hipGraphClone(&c, g));
  hipGraphNode_t keep;
  GX_CHECK(hipGraphNodeFindInClone(&keep, node, c));
  size_t n = 0;
  GX_CHECK(hipGraphGetNodes(c, nullptr, &n));
  std::vector<hipGraphNode_t> all(n);
  if (n) GX_CHECK(hipGraphGetNodes(c, all.data(), &n));
  for (auto x : all)
    if (x != keep) GX_CHECK(hipGraphDestroyNode(x));
  hipGraphExec_t e;
  GX_CHECK(hipGraphInstantiate(&e, c, nullptr, nullptr, 0));
  GX_CHECK(hipGraphDestroy(c));
  return e;
}

int64_t gexec_create(int64_t graph_handle, int64_t max_streams) {
  TORCH_CHECK(graph_handle != 0, "graphexec: null graph");
  TORCH_CHECK(max_streams >= 1 && max_streams <= 8, "graphexec: 1..8 streams");
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph_handle);
  size_t n = 0;
  GX_CHECK(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> raw(n);
  if (n) GX_CHECK(hipGraphGetNodes(g, raw.data(), &n));
  std::unordered_map<hipGraphNode_t, int> idx;
  for (size_t i = 0; i < n; ++i) idx[raw[i]] = (int)i;
  std::vector<std::vector<int>> parents(n), children(n);
  for (size_t i = 0; i < n; ++i) {
    size_t nd = 0;
    GX_CHECK(hipGraphNodeGetDependencies(raw[i], nullptr, &nd));
    std::vector<hipGraphNode_t> deps(nd);
    if (nd) GX_CHECK(hipGraphNodeGetDependencies(raw[i], deps.data(), &nd));
    for (auto d : deps) {
      auto it = idx.find(d);
      TORCH_CHECK(it != idx.end(), "graphexec: dependency outside the graph");
      parents[i].push_back(it->second);
      children[it->second].push_back((int)i);
    }
  }
  // topological order, ties broken by creation index (= capture order)
  std::vector<int> indeg(n), topo;
  topo.reserve(n);
  std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
  for (size_t i = 0; i < n; ++i) {
    indeg[i] = (int)parents[i].size();
    if (!indeg[i]) ready.push((int)i);
  }
  while (!ready.empty()) {
    int v = ready.top();
    ready.pop();
    topo.push_back(v);
    for (int c : children[v])
      if (--indeg[c] == 0) ready.push(c);
  }
  TORCH_CHECK(topo.size() == n, "graphexec: graph has a cycle");
  std::vector<int> pos(n);
  for (size_t i = 0; i < n; ++i) pos[topo[i]] = (int)i;

  auto ex = std::make_unique<Exec>();
  ex->nodes.resize(n);
  ex->par.assign(n, {});
  const int K = (int)max_streams;
  // ancestor sets as bitsets over topo positions (n is a few thousand at most)
  const size_t words = (n + 63) / 64;
  std::vector<uint64_t> anc(n * words, 0);
  auto is_anc = [&](int a_pos, int v_pos) {
    return (anc[(size_t)v_pos * words + a_pos / 64] >> (a_pos % 64)) & 1ull;
  };
  // heir of every node: the child that continues its stream — the one with the longest path
  // to the end of the graph (the critical chain, hundreds of nodes, not a weight-gradient
  // branch of two that ends at the final join), ties by capture order.  The other children
  // start on other streams, behind an event.  Continuing whichever child was captured first
  // put e.g. the downsample branch on the main chain's stream and moved the chain itself
  // behind an event (~20 µs of dependency latency at every such fork).
  std::vector<int> blevel(n, 0), heir(n, -1);
  for (size_t q = n; q-- > 0;) {
    const int v = topo[q];
    int best = 0;
    for (int c : children[v]) {
      const int cp = pos[c];
      if (heir[q] < 0 || blevel[cp] > best || (blevel[cp] == best && cp < heir[q])) {
        best = blevel[cp];
        heir[q] = cp;
      }
    }
    blevel[q] = 1 + best;
  }
  std::vector<int> tail(K, -1);      // topo position of each stream's last node
  std::vector<int> seq(n, 0);        // position of the node within its stream (1-based)
  std::vector<int> slen(K, 0);
  // vector clocks: clk[s][t] = last position on stream t that stream s already follows
  std::vector<std::vector<int>> clk(K, std::vector<int>(K, 0));
  std::vector<std::vector<int>> node_clk(n);
  int used = 1;
  for (size_t p = 0; p < n; ++p) {
    int v = topo[p];
    uint64_t* av = &anc[p * words];
    for (int u : parents[v]) {
      int up = pos[u];
      const uint64_t* au = &anc[(size_t)up * words];
      for (size_t w = 0; w < words; ++w) av[w] |= au[w];
      av[up / 64] |= 1ull << (up % 64);
    }
    // stream choice: (1) the stream of a parent whose heir this node is; (2) a stream whose
    // tail is an ancestor and not a parent still waiting for its heir (reserved); (3) a new one;
    // (4) a reserved ancestor stream; (5) the earliest tail (all streams run concurrent work)
    int s = -1;
    for (int u : parents[v]) {
      const int up = pos[u];
      if (heir[up] != (int)p) continue;
      for (int k = 0; k < used && s < 0; ++k)
        if (tail[k] == up) s = k;
      if (s >= 0) break;
    }
    // a stream whose tail is a parent of this node (which is not that parent's heir: else (1)
    // took it) is kept for the parent's heir, which comes later in capture order
    auto reserved = [&](int k) {
      if (tail[k] < 0 || heir[tail[k]] <= (int)p) return false;
      for (int u : parents[v])
        if (pos[u] == tail[k]) return true;
      return false;
    };
    if (s < 0)
      for (int k = 0; k < used && s < 0; ++k)
        if ((tail[k] < 0 || is_anc(tail[k], (int)p)) && !reserved(k)) s = k;
    if (s < 0 && used < K) s = used++;
    if (s < 0)
      for (int k = 0; k < used && s < 0; ++k)
        if (tail[k] < 0 || is_anc(tail[k], (int)p)) s = k;
    if (s < 0) {
      s = 0;
      for (int k = 1; k < used; ++k)
        if (tail[k] < tail[s]) s = k;
    }
    Node& nd = ex->nodes[p];
    nd.stream = s;
    for (int u : parents[v]) ex->par[p].push_back(pos[u]);
    // waits: parents on other streams that stream s does not already follow
    for (int u : parents[v]) {
      int up = pos[u];
      int su = ex->nodes[up].stream;
      if (su == s) continue;
      if (clk[s][su] >= seq[up]) continue;
      nd.waits.push_back(up);
      const auto& uc = node_clk[up];
      for (int k = 0; k < K; ++k) clk[s][k] = std::max(clk[s][k], uc[k]);
    }
    seq[p] = ++slen[s];
    clk[s][s] = seq[p];
    node_clk[p] = clk[s];
    tail[s] = (int)p;
  }
  ex->nstreams = used;
  // the busiest chain (the step's critical path: the dgrad / BatchNorm chain, not the weight
  // gradients beside it) becomes stream 0, the caller's stream.  (Replaying that chain on a
  // highest-priority stream instead was measured 27.9 vs 21.5 ms/step: rejected, r5 log.)
  {
    std::vector<int> cnt(used, 0);
    for (const Node& nd : ex->nodes) cnt[nd.stream]++;
    const int top = (int)(std::max_element(cnt.begin(), cnt.end()) - cnt.begin());
    if (top != 0)
      for (Node& nd : ex->nodes) nd.stream = nd.stream == top ? 0 : nd.stream == 0 ? top : nd.stream;
  }
  // node parameters
  for (size_t p = 0; p < n; ++p) {
    Node& nd = ex->nodes[p];
    hipGraphNode_t h = raw[topo[p]];
    hipGraphNodeType t;
    GX_CHECK(hipGraphNodeGetType(h, &t));
    switch (t) {
      case hipGraphNodeTypeKernel:
        nd.kind = kKernel;
        GX_CHECK(hipGraphKernelNodeGetParams(h, &nd.kp));
        TORCH_CHECK(nd.kp.func != nullptr && (nd.kp.kernelParams != nullptr || nd.kp.extra == nullptr),
                    "graphexec: kernel node with `extra` launch arguments is not supported");
        break;
      case hipGraphNodeTypeMemset:
        nd.kind = kMemset;
        GX_CHECK(hipGraphMemsetNodeGetParams(h, &nd.mp));
        TORCH_CHECK(nd.mp.dst != nullptr && nd.mp.width > 0 &&
                        (nd.mp.elementSize == 1 || nd.mp.elementSize == 2 || nd.mp.elementSize == 4),
                    "graphexec: memset node without readable parameters");
        TORCH_CHECK(nd.mp.height <= 1 || nd.mp.elementSize == 1,
                    "graphexec: 2-D memset of elements wider than a byte");
        break;
      case hipGraphNodeTypeHost:
        nd.kind = kHost;
        GX_CHECK(hipGraphHostNodeGetParams(h, &nd.hp));
        break;
      case hipGraphNodeTypeEmpty:
        nd.kind = kEmpty;
        break;
      case hipGraphNodeTypeEventRecord:
        nd.kind = kEvRecord;
        GX_CHECK(hipGraphEventRecordNodeGetEvent(h, &nd.ext_event));
        break;
      case hipGraphNodeTypeWaitEvent:
        nd.kind = kEvWait;
        GX_CHECK(hipGraphEventWaitNodeGetEvent(h, &nd.ext_event));
        break;
      default:  // memcpy, child graph, ...: a one-node graph of its own
        nd.kind = kSub;
        nd.sub = single_node_exec(g, h);
        break;
    }
    ex->counts[nd.kind] += 1;
    ex->counts[7] += (int64_t)nd.waits.size();
  }
  for (auto& nd : ex->nodes)
    for (int w : nd.waits)
      if (ex->nodes[w].event < 0) {
        hipEvent_t e;
        GX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ex->nodes[w].event = (int)ex->events.size();
        ex->events.push_back(e);
      }
  ex->streams.assign(used, nullptr);
  for (int k = 1; k < used; ++k) {
    GX_CHECK(hipStreamCreateWithFlags(&ex->streams[k], hipStreamNonBlocking));
    hipEvent_t e;
    GX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ex->joins.push_back(e);
  }
  GX_CHECK(hipEventCreateWithFlags(&ex->fork, hipEventDisableTiming));
  return reinterpret_cast<int64_t>(ex.release());
}

void issue(const Node& nd, hipStream_t st) {
  switch (nd.kind) {
    case kKernel:
      GX_CHECK(hipLaunchKernel(nd.kp.func, nd.kp.gridDim, nd.kp.blockDim, nd.kp.kernelParams,
                               nd.kp.sharedMemBytes, st));
      break;
    case kSub:
      GX_CHECK(hipGraphLaunch(nd.sub, st));
      break;
    case kMemset: {
      const hipMemsetParams& m = nd.mp;
      if (m.height > 1) {
        GX_CHECK(hipMemset2DAsync(m.dst, m.pitch, (int)m.value, m.width, m.height, st));
      } else if (m.elementSize == 1) {
        GX_CHECK(hipMemsetD8Async(m.dst, (unsigned char)m.value, m.width, st));
      } else if (m.elementSize == 2) {
        GX_CHECK(hipMemsetD16Async(m.dst, (unsigned short)m.value, m.width, st));
      } else {
        GX_CHECK(hipMemsetD32Async(m.dst, (int)m.value, m.width, st));
      }
      break;
    }
    case kHost:
      GX_CHECK(hipLaunchHostFunc(st, nd.hp.fn, nd.hp.userData));
      break;
    case kEvRecord:
      GX_CHECK(hipEventRecord(nd.ext_event, st));
      break;
    case kEvWait:
      GX_CHECK(hipStreamWaitEvent(st, nd.ext_event, 0));
      break;
    case kEmpty:
      break;
  }
}

void gexec_replay(int64_t h) {
  Exec* ex = as_exec(h);
  hipStream_t cur = at::hip::getCurrentHIPStream().stream();
  ex->streams[0] = cur;
  if (ex->nstreams > 1) {
    GX_CHECK(hipEventRecord(ex->fork, cur));
    for (int k = 1; k < ex->nstreams; ++k) GX_CHECK(hipStreamWaitEvent(ex->streams[k], ex->fork, 0));
  }
  for (const Node& nd : ex->nodes) {
    hipStream_t st = ex->streams[nd.stream];
    for (int w : nd.waits) GX_CHECK(hipStreamWaitEvent(st, ex->events[ex->nodes[w].event], 0));
    issue(nd, st);
    if (nd.event >= 0) GX_CHECK(hipEventRecord(ex->events[nd.event], st));
  }
  for (int k = 1; k < ex->nstreams; ++k) {
    GX_CHECK(hipEventRecord(ex->joins[k - 1], ex->streams[k]));
    GX_CHECK(hipStreamWaitEvent(cur, ex->joins[k - 1], 0));
  }
}

// One step issued serially on the caller's stream with a timing event after every node: the
// per-node durations (µs) for gexec_reschedule.  Executes the step once, like a replay.
std::vector<double> gexec_timed_replay(int64_t h) {
  Exec* ex = as_exec(h);
  hipStream_t cur = at::hip::getCurrentHIPStream().stream();
  const size_t n = ex->nodes.size();
  std::vector<hipEvent_t> ev(n + 1);
  for (auto& e : ev) GX_CHECK(hipEventCreate(&e));
  GX_CHECK(hipEventRecord(ev[0], cur));
  for (size_t i = 0; i < n; ++i) {
    issue(ex->nodes[i], cur);
    GX_CHECK(hipEventRecord(ev[i + 1], cur));
  }
  GX_CHECK(hipEventSynchronize(ev[n]));
  std::vector<double> d(n);
  for (size_t i = 0; i < n; ++i) {
    float ms = 0.f;
    GX_CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    d[i] = 1e3 * (double)ms;
  }
  for (auto e : ev) GX_CHECK(hipEventDestroy(e));
  return d;
}

// Re-plan the issue order and the stream of every node from measured node durations (list
// scheduling): simulate `max_streams` in-order streams, and repeatedly issue, among the nodes whose
// parents are issued, the one that can start earliest (a cross-stream parent costs `lat_us` of
// event latency; ties: the longer remaining path to the end of the step, then capture order) on
// the stream where it starts earliest (ties: the stream of its latest-finishing parent).  The
// capture-order heuristic of gexec_create queues a node behind an earlier-captured one on its
// stream even when that one becomes ready much later (e.g. a weight gradient behind one waiting
// for the dgrad chain); here every stream's order follows the simulated start times.  The busiest
// stream becomes stream 0.  Waits and events are rebuilt as in gexec_create.
// The list schedule itself (host-only, no HIP): parents per node in a valid topological order
// → (issue order, stream per node), the busiest stream renumbered 0.
void list_schedule(const std::vector<std::vector<int>>& parv, const std::vector<double>& dur,
                   int K, double lat_us, std::vector<int>& order, std::vector<int>& str) {
  const int n = (int)parv.size();
  std::vector<std::vector<int>> ch(n);
  for (int p = 0; p < n; ++p)
    for (int u : parv[p]) ch[u].push_back(p);
  std::vector<double> rank(n, 0.0);
  for (int p = n; p-- > 0;) {
    double best = 0.0;
    for (int c : ch[p]) best = std::max(best, rank[c]);
    rank[p] = std::max(dur[p], 0.0) + best;
  }
  std::vector<double> fin(n, 0.0), freeT(K, 0.0);
  std::vector<int> npar(n), ready;
  str.assign(n, -1);
  order.clear();
  order.reserve(n);
  for (int p = 0; p < n; ++p) {
    npar[p] = (int)parv[p].size();
    if (!npar[p]) ready.push_back(p);
  }
  while (!ready.empty()) {
    int bi = -1, bk = 0;
    double bt = 0.0;
    for (int i = 0; i < (int)ready.size(); ++i) {
      const int v = ready[i];
      int pref = -1;
      double pf = -1.0;
      for (int u : parv[v])
        if (fin[u] > pf) { pf = fin[u]; pref = str[u]; }
      int kk = -1;
      double tt = 0.0;
      for (int k = 0; k < K; ++k) {
        double t = freeT[k];
        for (int u : parv[v]) t = std::max(t, fin[u] + (str[u] == k ? 0.0 : lat_us));
        if (kk < 0 || t < tt - 1e-9 || (t <= tt + 1e-9 && k == pref)) { kk = k; tt = t; }
      }
      const int b = bi < 0 ? -1 : ready[bi];
      if (bi < 0 || tt < bt - 1e-9 ||
          (tt <= bt + 1e-9 && (rank[v] > rank[b] + 1e-9 || (rank[v] >= rank[b] - 1e-9 && v < b)))) {
        bi = i; bk = kk; bt = tt;
      }
    }
    const int v = ready[bi];
    ready.erase(ready.begin() + bi);
    str[v] = bk;
    fin[v] = bt + std::max(dur[v], 0.0);
    freeT[bk] = fin[v];
    order.push_back(v);
    for (int c : ch[v])
      if (--npar[c] == 0) ready.push_back(c);
  }
  TORCH_CHECK((int)order.size() == n, "graphexec: list schedule lost nodes (not a DAG?)");
  int used = 1;
  for (int p = 0; p < n; ++p) used = std::max(used, str[p] + 1);
  std::vector<int> cnt(used, 0);
  for (int p = 0; p < n; ++p) cnt[str[p]]++;
  const int top = (int)(std::max_element(cnt.begin(), cnt.end()) - cnt.begin());
  if (top != 0)
    for (int p = 0; p < n; ++p) str[p] = str[p] == top ? 0 : str[p] == 0 ? top : str[p];
}

void gexec_reschedule(int64_t h, std::vector<double> dur, int64_t max_streams, double lat_us) {
  Exec* ex = as_exec(h);
  const int n = (int)ex->nodes.size();
  TORCH_CHECK((int)dur.size() == n, "graphexec: one duration per node");
  TORCH_CHECK(max_streams >= 1 && max_streams <= 8, "graphexec: 1..8 streams");
  std::vector<int> order, str;
  list_schedule(ex->par, dur, (int)max_streams, lat_us, order, str);
  int used = 1;
  for (int p = 0; p < n; ++p) used = std::max(used, str[p] + 1);
  // rebuild the node list in the new order with waits pruned by vector clocks
  std::vector<int> npos(n);
  for (int q = 0; q < n; ++q) npos[order[q]] = q;
  std::vector<Node> nodes(n);
  std::vector<std::vector<int>> par(n);
  std::vector<int> seq(n, 0), slen(used, 0);
  std::vector<std::vector<int>> clk(used, std::vector<int>(used, 0)), node_clk(n);
  ex->counts[7] = 0;
  for (int q = 0; q < n; ++q) {
    const int v = order[q];
    Node nd = ex->nodes[v];
    nd.stream = str[v];
    nd.waits.clear();
    nd.event = -1;
    const int s = nd.stream;
    for (int u : ex->par[v]) par[q].push_back(npos[u]);
    for (int up : par[q]) {
      const int su = nodes[up].stream;
      if (su == s || clk[s][su] >= seq[up]) continue;
      nd.waits.push_back(up);
      for (int k = 0; k < used; ++k) clk[s][k] = std::max(clk[s][k], node_clk[up][k]);
    }
    seq[q] = ++slen[s];
    clk[s][s] = seq[q];
    node_clk[q] = clk[s];
    ex->counts[7] += (int64_t)nd.waits.size();
    nodes[q] = nd;
  }
  for (auto e : ex->events) GX_CHECK(hipEventDestroy(e));
  ex->events.clear();
  for (auto& nd : nodes)
    for (int w : nd.waits)
      if (nodes[w].event < 0) {
        hipEvent_t e;
        GX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        nodes[w].event = (int)ex->events.size();
        ex->events.push_back(e);
      }
  // the sub-graph executables move with their nodes (ownership stays with ex->nodes)
  ex->nodes.swap(nodes);
  for (auto& nd : nodes) nd.sub = nullptr;
  ex->par.swap(par);
  while ((int)ex->streams.size() < used) {
    hipStream_t st;
    GX_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    ex->streams.push_back(st);
    hipEvent_t e;
    GX_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ex->joins.push_back(e);
  }
  ex->nstreams = std::max(ex->nstreams, used);
}

// list_schedule on a DAG given as CSR parent lists (tests): [order..., stream per node...]
std::vector<int64_t> gexec_list_schedule_op(std::vector<int64_t> off, std::vector<int64_t> parents,
                                            std::vector<double> dur, int64_t max_streams,
                                            double lat_us) {
  const int n = (int)dur.size();
  TORCH_CHECK((int)off.size() == n + 1 && off[n] == (int64_t)parents.size(), "bad CSR");
  std::vector<std::vector<int>> parv(n);
  for (int p = 0; p < n; ++p)
    for (int64_t i = off[p]; i < off[p + 1]; ++i) {
      TORCH_CHECK(parents[i] >= 0 && parents[i] < p, "parents must precede their children");
      parv[p].push_back((int)parents[i]);
    }
  std::vector<int> order, str;
  list_schedule(parv, dur, (int)max_streams, lat_us, order, str);
  std::vector<int64_t> out(order.begin(), order.end());
  out.insert(out.end(), str.begin(), str.end());
  return out;
}

// [kernels, one-node sub-graphs, memsets, host, empty, event-record, event-wait, cross-stream
//  waits, streams, recorded events]
std::vector<int64_t> gexec_stats(int64_t h) {
  Exec* ex = as_exec(h);
  std::vector<int64_t> out(ex->counts, ex->counts + 8);
  out.push_back(ex->nstreams);
  out.push_back((int64_t)ex->events.size());
  return out;
}

// per issued node: stream index (tests / tools: the schedule the heuristic produced)
std::vector<int64_t> gexec_streams(int64_t h) {
  Exec* ex = as_exec(h);
  std::vector<int64_t> out;
  out.reserve(ex->nodes.size());
  for (const Node& nd : ex->nodes) out.push_back(nd.stream * 16 + (int64_t)nd.kind);
  return out;
}

void gexec_destroy(int64_t h) {
  if (h) delete as_exec(h);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(simclr_amd, m) {
  m.def("gexec_create(int graph, int max_streams) -> int", &gexec_create);
  m.def("gexec_replay(int handle) -> ()", &gexec_replay);
  m.def("gexec_stats(int handle) -> int[]", &gexec_stats);
  m.def("gexec_streams(int handle) -> int[]", &gexec_streams);
  m.def("gexec_destroy(int handle) -> ()", &gexec_destroy);
  m.def("gexec_timed_replay(int handle) -> float[]", &gexec_timed_replay);
  m.def("gexec_list_schedule(int[] offsets, int[] parents, float[] durations, int max_streams, "
        "float lat_us) -> int[]", &gexec_list_schedule_op);
  m.def("gexec_reschedule(int handle, float[] durations, int max_streams, float lat_us) -> ()",
        &gexec_reschedule);
}

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
}

// ws_loopback.hpp -- live loopback websocket echo server + the ping-pong
// client of benchmarks/bench-websocket-pingpong.sh (C1), in one process, with
// the server's frame decoder as a template parameter:
//
//   gev_amd/ws_loopback      DeviceDecoder (ws_loopback.cpp): one device pass
//                            per loop iteration over every readable upgraded
//                            connection (gevws_protocol_unpacket_batch), then
//                            UnPacket per connection -- the product path.
//   tools/ws_loopback_cpu    the CPU baseline beside it: the reference's
//                            per-frame UnPacket pipeline restated in
//                            oracle/ws_ref.c (header parse, make, ring Read,
//                            Cipher) on the loop's own core.  Never linked into
//                            libgevws.so or gev_amd/ws_loopback.
//
// Server, shaped like gev: L event loops (eventloop.go), each with its own
// epoll, SO_REUSEPORT listener and decoder (one context + protocol per loop,
// thread-confined), and per connection a gevws_conn + gevws_ring
// (connection.go).  One loop iteration = epoll_wait -> one read(2) of <= 64 KiB
// per readable connection into its ring (handleRead, connection.go:220-251;
// eventloop.go:15) -> decoder pass -> per connection UnPacket until (nil, nil)
// (handlerProtocol, connection.go:208-218), answering the handshake
// (gevws_upgrader, ws.go:158-343) and echoing every data frame as a binary
// frame (benchmarks/websocket/server.go:22-29, ws.NewBinaryFrame +
// FrameToBytes) -> write(2).  Partial frames stay in the ring for the next
// pass (the streaming carry across batches).
//
// Client: C connections spread over T threads; each does the upgrade, then
// sends one masked text frame of M random bytes, waits for the echo, checks it
// byte for byte, repeats for the run time.
//
// --mode wsserver mirrors the reference's own end-to-end test,
// example/websocket/wsserver_test.go:73-133 with wsExample (:22-70): every
// client sends masked text frames of random 1..3072 bytes and reads the same
// number of bytes back (io.ReadFull + bytes.Equal); the server's OnMessage
// answers (MessageText, data) either by return value or by c.Send(PackData)
// at random (:47-63) -- here every frame's reply is computed on the device by
// the protocol's handler step (HandlerWrap.OnMessage + FrameToBytes,
// gevws_protocol_set_handler(GEVWS_HANDLER_ECHO_TEXT)) and routed either into
// the returned `out` (sent after the connection's handlerProtocol) or into a
// queue sent after the loop iteration (c.Send -> QueueInLoop).  --ctrl P
// precedes a message with a masked ping (or pong) with probability P; the
// device's control reply (pong / the reference's ping-for-pong) is returned
// inline; --close-end 1 ends every client with a close frame (valid, reserved,
// unknown and application codes; UTF-8 and invalid reasons; empty bodies),
// answered by util.HandleClose's reply plus ShutdownWrite (wrap.go:45-68), so
// the client must see the reply and then EOF.  --transcript FILE writes every
// (control frame sent, reply received) pair as hex for the oracle check
// (tests/test_gpu_loopback.py against oracle/ws_oracle.on_message).
//
// --mode close mirrors TestWebSocketServer_CloseConnection
// (wsserver_test.go:135-178): --conns clients dial and upgrade, --to-close of
// them close (a close frame first with --close-frame 1, as x/net/websocket's
// Conn.Close; a bare TCP close with 0), and the server's OnConnect - OnClose
// count must be conns - to_close after the drain, then 0 once the rest close.
//
//   [--conns 1000] [--msg 128] [--seconds 5] [--loops 1] [--client-threads 4]
//   [--port 0] [--device 0] [--mode echo|wsserver] [--ctrl 0] [--close-end 0]
//   [--transcript FILE] [--seed 1] [--devices 1]
// --devices N places loop l on device (--device + l % N): the loops of one
// server process spread over the node's GPUs round-robin, each with its own
// context and protocol (a connection stays on its loop's GPU).
// Prints one JSON line.
#pragma once

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <deque>
#include <mutex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gevws.h"

namespace wslb {

inline std::atomic<bool> g_stop{false};
inline std::atomic<uint64_t> g_batches{0}, g_batch_conns{0}, g_frames{0}, g_bad{0}, g_dev_ns{0};
// frames echoed per server loop (fairness across loops: "loop_echoes_per_s")
constexpr int kMaxLoops = 64;
inline std::atomic<uint64_t> g_loop_frames[kMaxLoops];
inline std::atomic<uint64_t> g_loop_conns[kMaxLoops];  // connections accepted per loop (SO_REUSEPORT hashing)
// every loop's decoders' pass timelines (Decoder::kTimeline), summed at loop exit
inline std::mutex g_tl_mu;
inline gevws_protocol_timeline g_tl{};
inline std::atomic<uint64_t> g_service_passes{0};  // of those, posted to a resident decode service
inline std::atomic<uint64_t> g_direct_passes{0};   // ... written into a context's own AQL queue
inline void add_timeline(const gevws_protocol_timeline& t) {
  std::lock_guard<std::mutex> g(g_tl_mu);
  g_tl.passes += t.passes;
  g_tl.signalled += t.signalled;
  g_tl.ns_select += t.ns_select;
  g_tl.ns_stage += t.ns_stage;
  g_tl.ns_launch += t.ns_launch;
  g_tl.ns_wait += t.ns_wait;
  g_tl.ns_deliver += t.ns_deliver;
  g_tl.ns_gpu_decode += t.ns_gpu_decode;
  g_tl.ns_gpu_handler += t.ns_gpu_handler;
  g_tl.ns_gpu_gap += t.ns_gpu_gap;
}
inline std::atomic<uint64_t> g_ctrl{0}, g_closed{0}, g_sent_async{0}, g_payload{0};
// OnConnect / OnClose of every server loop (wsExample.ClientNum,
// example/websocket/wsserver_test.go:22-45): +1 at accept, -1 when the loop
// closes the connection (EOF or error on read, connection.go:288-303)
inline std::atomic<int64_t> g_live{0};

enum { kModeEcho = 0, kModeWsServer = 1, kModeClose = 2 };
struct Config {
  int mode = kModeEcho;
  double ctrl_prob = 0.0;  // wsserver: a control frame before a message with this probability
  bool close_end = false;  // wsserver: every client ends with a close frame
  int to_close = 5;         // close mode: connections the client closes
  bool close_frame = true;  // close mode: a close frame before the TCP close (x/net/websocket Conn.Close)
  std::string transcript;  // wsserver: (control frame sent, reply) pairs, hex
  unsigned seed = 1;
};
inline Config g_cfg;
inline std::mutex g_tr_mu;
inline std::vector<std::pair<std::vector<uint8_t>, std::vector<uint8_t>>> g_transcript;

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

// ws.WriteHeader (write.go:48-84) for a server frame (unmasked).
inline uint32_t write_header(uint8_t* o, uint8_t b0, uint64_t len) {
  o[0] = b0;
  if (len <= 125) {
    o[1] = (uint8_t)len;
    return 2;
  }
  if (len <= 0xFFFF) {
    o[1] = 126;
    o[2] = (uint8_t)(len >> 8);
    o[3] = (uint8_t)len;
    return 4;
  }
  o[1] = 127;
  for (int i = 0; i < 8; ++i) o[2 + i] = (uint8_t)(len >> (56 - 8 * i));
  return 10;
}

inline bool send_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EAGAIN || errno == EINTR) continue;  // loopback: the peer drains promptly
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

// ------------------------------------------------------------------ server
struct ServerConn {
  int fd;
  gevws_conn* c;
  gevws_ring* r;
  std::vector<uint8_t> out;
  std::vector<uint8_t> frame;  // CpuDecoder: the payload slice it returned last (Go's make)
  int poisoned = 0;
  std::vector<uint8_t> queued;  // wsserver: c.Send(PackData(...)) output, sent after the loop iteration
  bool shut = false;            // wsserver: ShutdownWrite done (a close was answered)
  int half = 0;                 // split passes: which of the loop's two decoders owns it
};

// Decoder concept:
//   explicit Decoder(int device);
//   int64_t pass(ServerConn* const* conns, uint32_t n);   // readable upgraded connections
//   int unpacket(ServerConn* s, gevws_header* h, const uint8_t** data, uint64_t* len);
//   static const char* name();
//   static constexpr bool kHandler;  // reply(): HandlerWrap.OnMessage's answer for the last frame
//   void set_handler(int policy);
//   int reply(ServerConn* s, const uint8_t** out, uint64_t* len, int* shutdown_write);
template <class Decoder>
void server_loop(int port, int device, std::atomic<int>* ready, int index) {
  Decoder dec(device);
  const bool wss = g_cfg.mode != kModeEcho;
  if (wss) dec.set_handler(GEVWS_HANDLER_ECHO_TEXT);  // wsExample.OnMessage returns (MessageText, data)
  // GEVWS_LB_SPLIT=K (a pipelined decoder; default 64, 0 = off): an
  // iteration with at least K readable connections makes W = GEVWS_LB_WAYS
  // (default 2, at most 8) device passes, each on its own decoder
  // (connections are dealt to them at accept): group g's pass runs while
  // groups g+1.. are read and groups ..g-1 are echoed -- every echo still goes
  // out in the iteration that read its frame.  100 connections on one loop:
  // 461-463 k -> 482-493 k echoes/s with two groups, 3 or 4 no better
  // (profiles/r04/r04_loopback_split_ways.jsonl).
  const char* se = getenv("GEVWS_LB_SPLIT");
  const uint32_t split_min = Decoder::kPipelined ? (se ? (uint32_t)strtoul(se, nullptr, 10) : 64u) : 0u;
  const char* we = getenv("GEVWS_LB_WAYS");
  const uint32_t ways = split_min ? std::min(8u, std::max(2u, we ? (uint32_t)strtoul(we, nullptr, 10) : 2u)) : 1u;
  std::vector<std::unique_ptr<Decoder>> decs;  // groups 1 .. ways-1 (group 0: dec)
  for (uint32_t g = 1; g < ways; ++g) {
    decs.emplace_back(new Decoder(device));
    if (wss) decs.back()->set_handler(GEVWS_HANDLER_ECHO_TEXT);
  }
  auto dec_of = [&](uint32_t g) -> Decoder& { return g == 0 ? dec : *decs[g - 1]; };
  uint32_t accepted = 0;
  std::mt19937_64 route(g_cfg.seed * 1000003u + (unsigned)index);  // wsserver_test.go:47: rand.Int() % 2
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  setsockopt(ls, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (bind(ls, (sockaddr*)&a, sizeof(a)) || listen(ls, 4096)) {
    perror("ws_loopback: bind/listen");
    exit(2);
  }
  set_nonblock(ls);
  int ep = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = ls;
  epoll_ctl(ep, EPOLL_CTL_ADD, ls, &ev);
  ready->fetch_add(1);

  std::unordered_map<int, ServerConn> conns;
  std::vector<epoll_event> evs(4096);
  std::vector<uint8_t> rbuf(65536);  // the loop's packet buffer (eventloop.go:15)
  std::vector<ServerConn*> readable, upgraded, inflight;
  // GEVWS_LB_PIPELINE=1 with a pipelined decoder (Decoder::kPipelined): the
  // device pass of iteration k runs while iteration k+1 waits on epoll and
  // reads its sockets, and its frames are echoed after those reads.  Measured
  // slower than the serial loop (pass, then echo) with closed-loop clients
  // (profiles/r02/r02_loopback_pipeline_ab.jsonl): a connection only sends again
  // once echoed, so the overlap splits the connections into two alternating
  // passes of half the size, twice the fixed cost per pass -- default off.
  const char* pe = getenv("GEVWS_LB_PIPELINE");
  const bool pipeline = Decoder::kPipelined && pe && atoi(pe) == 1;
  bool pending = false;
  // handlerProtocol for one connection: UnPacket until (nil, nil), echo
  std::vector<ServerConn*> queued_conns;
  auto handle_with = [&](Decoder& dec, ServerConn* s, double& t_dec) {
    s->out.clear();
    bool shut = false;
    for (;;) {
      gevws_header h;
      const uint8_t* data = nullptr;
      uint64_t len = 0;
      const double tu = now_s();
      const int st = dec.unpacket(s, &h, &data, &len);
      t_dec += now_s() - tu;
      if (st == GEVWS_OK && wss) {
        // HandlerWrap.OnMessage (wrap.go:38-90): the device handler's reply
        const uint8_t* rp = nullptr;
        uint64_t rl = 0;
        int sh = 0;
        std::vector<uint8_t> host_reply;
        if constexpr (Decoder::kHandler) {
          if (dec.reply(s, &rp, &rl, &sh) != GEVWS_OK) g_bad.fetch_add(1);
        } else if (!(h.opcode & 0x8) && len) {  // CPU twin: data frames only, echoed as text on the host
          uint8_t hdr[14];
          const uint32_t hn = write_header(hdr, 0x81, len);
          host_reply.assign(hdr, hdr + hn);
          host_reply.insert(host_reply.end(), data, data + len);
          rp = host_reply.data();
          rl = host_reply.size();
        }
        if (h.opcode & 0x8) {  // control: HandlerWrap returns the reply (sent with handlerProtocol's out)
          s->out.insert(s->out.end(), rp, rp + rl);
          shut = shut || sh;
          g_ctrl.fetch_add(1, std::memory_order_relaxed);
        } else {
          if (route() & 1) {  // case 1: c.Send(util.PackData(ws.MessageText, data)) -> QueueInLoop
            if (s->queued.empty()) queued_conns.push_back(s);
            s->queued.insert(s->queued.end(), rp, rp + rl);
            g_sent_async.fetch_add(1, std::memory_order_relaxed);
          } else {  // case 0: out = data, framed by HandlerWrap (NewTextFrame + FrameToBytes)
            s->out.insert(s->out.end(), rp, rp + rl);
          }
          g_frames.fetch_add(1, std::memory_order_relaxed);
          g_loop_frames[index % kMaxLoops].fetch_add(1, std::memory_order_relaxed);
          g_payload.fetch_add(len, std::memory_order_relaxed);
        }
      } else if (st == GEVWS_OK) {
        if (h.opcode & 0x8) continue;  // control frames: not in this workload
        uint8_t hdr[14];
        const uint32_t hn = write_header(hdr, 0x82, len);  // NewBinaryFrame + FrameToBytes
        s->out.insert(s->out.end(), hdr, hdr + hn);
        s->out.insert(s->out.end(), data, data + len);
        g_frames.fetch_add(1, std::memory_order_relaxed);
        g_loop_frames[index % kMaxLoops].fetch_add(1, std::memory_order_relaxed);
        g_payload.fetch_add(len, std::memory_order_relaxed);
      } else if (len != 0) {
        s->out.insert(s->out.end(), data, data + len);  // handshake response (wrap.go:40-42)
      } else {
        break;
      }
    }
    // (close mode: the peer may already be gone when its close reply goes out;
    // gev then just closes the connection, connection.go:305-328)
    if (!s->out.empty() && !s->shut && !send_all(s->fd, s->out.data(), s->out.size()) && g_cfg.mode != kModeClose)
      g_bad.fetch_add(1);
    if (shut && !s->shut) {  // c.ShutdownWrite() after the close reply (wrap.go:56)
      ::shutdown(s->fd, SHUT_WR);
      s->shut = true;
      g_closed.fetch_add(1, std::memory_order_relaxed);
    }
  };
  // the loop's pending functions (doPendingFunc): the c.Send calls of this iteration
  auto flush_queued = [&]() {
    for (ServerConn* s : queued_conns) {
      if (!s->shut && !s->queued.empty() && !send_all(s->fd, s->queued.data(), s->queued.size())) g_bad.fetch_add(1);
      s->queued.clear();
    }
    queued_conns.clear();
  };
  auto handle = [&](ServerConn* s, double& t_dec) { handle_with(dec, s, t_dec); };
  // the pass in flight, ended and its frames handed out (also before a
  // connection it holds is closed: the protocol writes to its rings' owners)
  auto finish = [&](double& t_dec) {
    if (!pending) return;
    const double td = now_s();
    const int64_t f = dec.end();
    t_dec += now_s() - td;
    if (f < 0) {
      fprintf(stderr, "ws_loopback: decoder pass %s\n", gevws_status_string((int)f));
      exit(3);
    }
    pending = false;
    for (ServerConn* s : inflight) handle(s, t_dec);
  };
  double t_close = 0;
  std::vector<std::vector<int>> deferred(ways);     // split: groups 1.. readable fds
  std::vector<std::vector<ServerConn*>> rd(ways), up(ways);
  while (!g_stop.load(std::memory_order_relaxed)) {
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), pending ? 0 : 5);
    readable.clear();
    for (auto& d : deferred) d.clear();
    // one read(2) per readable connection (handleRead), its bytes into the ring
    auto read_conn = [&](int fd, std::vector<ServerConn*>& into) {
      auto it = conns.find(fd);
      if (it == conns.end()) return;
      const ssize_t k = ::read(fd, rbuf.data(), rbuf.size());
      if (k <= 0) {
        if (k < 0 && (errno == EAGAIN || errno == EINTR)) return;
        finish(t_close);
        flush_queued();
        epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
        close(fd);
        gevws_conn_free(it->second.c);
        gevws_ring_free(it->second.r);
        conns.erase(it);
        g_live.fetch_sub(1);  // OnClose
        return;
      }
      gevws_ring_write(it->second.r, rbuf.data(), (uint64_t)k);
      into.push_back(&it->second);
    };
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd != ls && split_min) {
        auto it = conns.find(fd);
        if (it != conns.end() && it->second.half != 0) {  // read after the earlier groups' passes are launched
          deferred[it->second.half].push_back(fd);
          continue;
        }
      }
      if (fd == ls) {
        for (;;) {
          int cfd = accept4(ls, nullptr, nullptr, SOCK_NONBLOCK);
          if (cfd < 0) break;
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          ServerConn sc{cfd, gevws_conn_new(), gevws_ring_new(4096), {}, {}, 0};  // DefaultBufferSize
          sc.half = split_min ? (int)(accepted++ % ways) : 0;
          gevws_conn_set_upgraded(sc.c, 0);
          conns.emplace(cfd, std::move(sc));
          g_live.fetch_add(1);  // OnConnect
          g_loop_conns[index % kMaxLoops].fetch_add(1, std::memory_order_relaxed);
          epoll_event ce{};
          ce.events = EPOLLIN;
          ce.data.fd = cfd;
          epoll_ctl(ep, EPOLL_CTL_ADD, cfd, &ce);
        }
        continue;
      }
      read_conn(fd, readable);
    }
    // decode time of the iteration: the pass plus the UnPacket calls (the
    // device decoder's UnPacket only pops queued frames; the CPU decoder's
    // does the whole per-frame pipeline), not the echo's encode or write(2)
    double t_dec = t_close;
    t_close = 0;
    finish(t_dec);  // the pass begun last iteration: its frames go out now
    size_t nready = readable.size();
    for (auto& d : deferred) nready += d.size();
    if (split_min && !pipeline && nready >= split_min) {  // (not with GEVWS_LB_PIPELINE)
      // W passes: group g's begins once its sockets are read, ends once the
      // groups after it are read and the groups before it echoed
      auto begin_group = [&](Decoder& d, std::vector<ServerConn*>& rg, std::vector<ServerConn*>& ug) -> bool {
        ug.clear();
        for (ServerConn* s : rg)
          if (gevws_conn_upgraded(s->c)) ug.push_back(s);
        if (ug.empty()) return false;
        const double td = now_s();
        const int64_t f = d.begin(ug.data(), (uint32_t)ug.size());
        t_dec += now_s() - td;
        if (f < 0) {
          fprintf(stderr, "ws_loopback: decoder pass %s\n", gevws_status_string((int)f));
          exit(3);
        }
        g_batches.fetch_add(1, std::memory_order_relaxed);
        g_batch_conns.fetch_add(ug.size(), std::memory_order_relaxed);
        return true;
      };
      auto end_group = [&](Decoder& d, bool began, std::vector<ServerConn*>& rg) {
        if (began) {
          const double td = now_s();
          const int64_t f = d.end();
          t_dec += now_s() - td;
          if (f < 0) {
            fprintf(stderr, "ws_loopback: decoder pass %s\n", gevws_status_string((int)f));
            exit(3);
          }
        }
        for (ServerConn* s : rg) handle_with(d, s, t_dec);  // (handshakes too)
      };
      bool began[8] = {};
      rd[0].swap(readable);
      for (uint32_t g = 0; g < ways; ++g) {
        if (g) {
          rd[g].clear();
          for (int fd : deferred[g]) read_conn(fd, rd[g]);
        }
        began[g] = begin_group(dec_of(g), rd[g], up[g]);
      }
      for (uint32_t g = 0; g < ways; ++g) end_group(dec_of(g), began[g], rd[g]);
      rd[0].swap(readable);
      flush_queued();
      g_dev_ns.fetch_add((uint64_t)(t_dec * 1e9), std::memory_order_relaxed);
      continue;
    }
    for (uint32_t g = 1; g < ways; ++g)
      for (int fd : deferred[g]) read_conn(fd, readable);  // (split on, a small iteration: one pass)
    if (readable.empty()) {
      flush_queued();
      g_dev_ns.fetch_add((uint64_t)(t_dec * 1e9), std::memory_order_relaxed);
      continue;
    }
    upgraded.clear();
    for (ServerConn* s : readable) {
      if (gevws_conn_upgraded(s->c)) upgraded.push_back(s);
      else if (pipeline) handle(s, t_dec);  // the handshake: no device pass involved
    }
    if (!upgraded.empty()) {
      const double td = now_s();
      const int64_t f = pipeline ? dec.begin(upgraded.data(), (uint32_t)upgraded.size())
                                 : dec.pass(upgraded.data(), (uint32_t)upgraded.size());
      t_dec += now_s() - td;
      if (f < 0) {
        fprintf(stderr, "ws_loopback: decoder pass %s\n", gevws_status_string((int)f));
        exit(3);
      }
      g_batches.fetch_add(1, std::memory_order_relaxed);
      g_batch_conns.fetch_add(upgraded.size(), std::memory_order_relaxed);
      if (pipeline && f > 0) {  // in flight: the next iteration reads its sockets meanwhile
        pending = true;
        inflight = upgraded;
      }
    }
    if (!pipeline)
      for (ServerConn* s : readable) handle(s, t_dec);  // handlerProtocol per connection
    flush_queued();
    g_dev_ns.fetch_add((uint64_t)(t_dec * 1e9), std::memory_order_relaxed);
  }
  if (pending) (void)dec.end();
  if constexpr (Decoder::kTimeline) {
    gevws_protocol_timeline t;
    dec.timeline(&t);
    add_timeline(t);
    for (auto& d : decs) {
      d->timeline(&t);
      add_timeline(t);
    }
  }
  decs.clear();
  for (auto& kv : conns) {
    close(kv.first);
    gevws_conn_free(kv.second.c);
    gevws_ring_free(kv.second.r);
  }
  close(ls);
  close(ep);
}

// ------------------------------------------------------------------ client
struct ClientConn {
  int fd;
  bool upgraded = false;
  std::vector<uint8_t> in;
  std::vector<uint8_t> sent;  // payload of the frame in flight
  uint64_t done = 0;
};

inline void client_send(ClientConn& c, std::mt19937_64& rng, size_t msg) {
  c.sent.resize(msg);
  for (auto& b : c.sent) b = (uint8_t)rng();
  std::vector<uint8_t> f(14 + msg);
  uint32_t hn = write_header(f.data(), 0x81, msg);  // masked text frame (x/net/websocket client)
  f[1] |= 0x80;
  const uint32_t key = (uint32_t)rng();
  uint8_t m[4];
  memcpy(m, &key, 4);
  memcpy(f.data() + hn, m, 4);
  hn += 4;
  for (size_t i = 0; i < msg; ++i) f[hn + i] = c.sent[i] ^ m[i & 3];
  if (!send_all(c.fd, f.data(), hn + msg)) g_bad.fetch_add(1);
}

inline void client_thread(int port, int nconn, size_t msg, double t_end, std::atomic<uint64_t>* total,
                          std::atomic<int>* upgraded_conns, unsigned seed) {
  std::mt19937_64 rng(seed);
  int ep = epoll_create1(0);
  std::vector<ClientConn> cs(nconn);
  const char req_fmt[] =
      "GET / HTTP/1.1\r\nHost: 127.0.0.1:%d\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
      "Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nOrigin: ws://127.0.0.1\r\nSec-WebSocket-Version: 13\r\n\r\n";
  char req[512];
  const int rn = snprintf(req, sizeof(req), req_fmt, port);
  for (int i = 0; i < nconn; ++i) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
      perror("ws_loopback: socket");
      _exit(2);
    }
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&a, sizeof(a))) {
      perror("ws_loopback: connect");
      _exit(2);  // other threads are running: no static destructors
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    set_nonblock(fd);
    cs[i].fd = fd;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
    send_all(fd, (const uint8_t*)req, (size_t)rn);
  }
  std::vector<epoll_event> evs(1024);
  std::vector<uint8_t> buf(1 << 16);
  while (now_s() < t_end && !g_stop.load(std::memory_order_relaxed)) {
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), 5);
    for (int e = 0; e < n; ++e) {
      ClientConn& c = cs[evs[e].data.u32];
      const ssize_t k = ::read(c.fd, buf.data(), buf.size());
      if (k <= 0) continue;
      c.in.insert(c.in.end(), buf.data(), buf.data() + k);
      if (!c.upgraded) {
        const std::string s(c.in.begin(), c.in.end());
        const size_t pos = s.find("\r\n\r\n");
        if (pos == std::string::npos) continue;
        if (s.compare(0, 12, "HTTP/1.1 101") != 0 || s.find("s3pPLMBiTxaQ9kYGzzhZRbK+xOo=") == std::string::npos) {
          g_bad.fetch_add(1);
          continue;
        }
        c.in.erase(c.in.begin(), c.in.begin() + (long)pos + 4);
        c.upgraded = true;
        upgraded_conns->fetch_add(1);
        client_send(c, rng, msg);
        continue;
      }
      // echo: unmasked binary frame carrying the same bytes
      const size_t hn = msg <= 125 ? 2 : (msg <= 0xFFFF ? 4 : 10);
      while (c.in.size() >= hn + msg) {
        if (c.in[0] != 0x82 || memcmp(c.in.data() + hn, c.sent.data(), msg) != 0) g_bad.fetch_add(1);
        c.in.erase(c.in.begin(), c.in.begin() + (long)(hn + msg));
        c.done++;
        client_send(c, rng, msg);
      }
    }
  }
  uint64_t sum = 0;
  for (auto& c : cs) {
    sum += c.done;
    close(c.fd);
  }
  total->fetch_add(sum);
  close(ep);
}

// ------------------------------------------------------------------ wsserver_test.go client
// startWebSocketClient (wsserver_test.go:101-133): masked text frames of
// 1..3072 random bytes, the echo read back in full and compared; optional
// control frames (--ctrl) before a message and a closing handshake at the end
// (--close-end).  Server frames are parsed as they arrive: text payload bytes
// accumulate until the message's length (io.ReadFull), control frames are
// paired with the control frame they answer (in order) for the transcript.
struct WsClient {
  int fd = -1;
  bool upgraded = false;
  int state = 0;  // 0 running, 1 close sent (reply + EOF expected), 2 done
  std::vector<uint8_t> in, data, got;
  std::deque<std::vector<uint8_t>> ctrl_sent;  // control frames awaiting their reply
  uint64_t done = 0;
};

inline std::vector<uint8_t> masked_frame(std::mt19937_64& rng, uint8_t b0, const uint8_t* p, size_t n) {
  std::vector<uint8_t> f(14 + n);
  uint32_t hn = write_header(f.data(), b0, n);
  f[1] |= 0x80;
  const uint32_t key = (uint32_t)rng();
  memcpy(f.data() + hn, &key, 4);
  const uint8_t* m = f.data() + hn;
  hn += 4;
  for (size_t i = 0; i < n; ++i) f[hn + i] = p[i] ^ m[i & 3];
  f.resize(hn + n);
  return f;
}

inline void ws_client_next(WsClient& c, std::mt19937_64& rng) {
  std::uniform_real_distribution<double> u(0.0, 1.0);
  if (g_cfg.ctrl_prob > 0 && u(rng) < g_cfg.ctrl_prob) {  // a ping (or a pong) before the message
    std::vector<uint8_t> p(rng() % 126);
    for (auto& b : p) b = (uint8_t)rng();
    auto f = masked_frame(rng, u(rng) < 0.8 ? 0x89 : 0x8A, p.data(), p.size());
    if (!send_all(c.fd, f.data(), f.size())) g_bad.fetch_add(1);
    c.ctrl_sent.push_back(std::move(f));
  }
  c.data.resize(rng() % (1024 * 3) + 1);  // wsserver_test.go:112
  for (auto& b : c.data) b = (uint8_t)rng();
  c.got.clear();
  auto f = masked_frame(rng, 0x81, c.data.data(), c.data.size());  // x/net/websocket: text frames
  if (!send_all(c.fd, f.data(), f.size())) g_bad.fetch_add(1);
}

inline void ws_client_close(WsClient& c, std::mt19937_64& rng) {
  static const uint16_t kCodes[] = {1000, 1001, 1002, 1003, 1005, 1006, 1007, 1011, 1015, 1016, 2999, 3000, 4999, 999};
  static const char* kReasons[] = {"", "bye", "normal closure", "\xc3\x28", "caf\xc3\xa9", "\xff"};
  std::vector<uint8_t> body;
  if (rng() % 8) {
    const uint16_t code = kCodes[rng() % (sizeof(kCodes) / sizeof(kCodes[0]))];
    body.push_back((uint8_t)(code >> 8));
    body.push_back((uint8_t)code);
    const char* r = kReasons[rng() % (sizeof(kReasons) / sizeof(kReasons[0]))];
    body.insert(body.end(), r, r + strlen(r));
  }
  auto f = masked_frame(rng, 0x88, body.data(), body.size());
  if (!send_all(c.fd, f.data(), f.size())) g_bad.fetch_add(1);
  c.ctrl_sent.push_back(std::move(f));
  c.state = 1;
}

inline void ws_client_thread(int port, int nconn, double t_end, std::atomic<uint64_t>* total,
                             std::atomic<int>* upgraded_conns, unsigned seed) {
  std::mt19937_64 rng(seed);
  int ep = epoll_create1(0);
  std::vector<WsClient> cs(nconn);
  std::vector<std::pair<std::vector<uint8_t>, std::vector<uint8_t>>> tr;
  const char req_fmt[] =
      "GET / HTTP/1.1\r\nHost: 127.0.0.1:%d\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
      "Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nOrigin: ws://127.0.0.1\r\nSec-WebSocket-Version: 13\r\n\r\n";
  char req[512];
  const int rn = snprintf(req, sizeof(req), req_fmt, port);
  for (int i = 0; i < nconn; ++i) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (fd < 0 || connect(fd, (sockaddr*)&a, sizeof(a))) {
      perror("ws_loopback: connect");
      _exit(2);
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    set_nonblock(fd);
    cs[i].fd = fd;
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
    send_all(fd, (const uint8_t*)req, (size_t)rn);
  }
  std::vector<epoll_event> evs(1024);
  std::vector<uint8_t> buf(1 << 16);
  const double t_hard = t_end + 5.0;  // closing handshakes must finish by then
  int finished = 0;
  while (!g_stop.load(std::memory_order_relaxed)) {
    const double now = now_s();
    if (now >= t_hard || (now >= t_end && (!g_cfg.close_end || finished == nconn))) break;
    const int n = epoll_wait(ep, evs.data(), (int)evs.size(), 5);
    for (int e = 0; e < n; ++e) {
      WsClient& c = cs[evs[e].data.u32];
      if (c.state == 2) continue;
      const ssize_t k = ::read(c.fd, buf.data(), buf.size());
      if (k == 0) {  // EOF: only after the close reply (the server's ShutdownWrite)
        if (c.state == 1 && c.ctrl_sent.empty()) {
          c.state = 2;
          ++finished;
          epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
        } else {
          g_bad.fetch_add(1);
          c.state = 2;
          ++finished;
          epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
        }
        continue;
      }
      if (k < 0) continue;
      c.in.insert(c.in.end(), buf.data(), buf.data() + k);
      if (!c.upgraded) {
        const std::string s(c.in.begin(), c.in.end());
        const size_t pos = s.find("\r\n\r\n");
        if (pos == std::string::npos) continue;
        if (s.compare(0, 12, "HTTP/1.1 101") != 0 || s.find("s3pPLMBiTxaQ9kYGzzhZRbK+xOo=") == std::string::npos) {
          g_bad.fetch_add(1);
          continue;
        }
        c.in.erase(c.in.begin(), c.in.begin() + (long)pos + 4);
        c.upgraded = true;
        upgraded_conns->fetch_add(1);
        ws_client_next(c, rng);
      }
      // server frames (unmasked)
      size_t off = 0;
      for (;;) {
        const size_t avail = c.in.size() - off;
        if (avail < 2) break;
        const uint8_t* f = c.in.data() + off;
        const uint32_t len7 = f[1] & 0x7f;
        const size_t hn = len7 < 126 ? 2 : (len7 == 126 ? 4 : 10);
        if (avail < hn) break;
        uint64_t L = len7;
        if (len7 == 126) L = ((uint64_t)f[2] << 8) | f[3];
        if (len7 == 127) {
          L = 0;
          for (int i = 0; i < 8; ++i) L = (L << 8) | f[2 + i];
        }
        if ((f[1] & 0x80) || avail - hn < L) {
          if (f[1] & 0x80) g_bad.fetch_add(1);  // a server frame must not be masked
          break;
        }
        if (f[0] & 0x08) {  // a control reply: pair it with the oldest unanswered control frame
          if (c.ctrl_sent.empty()) {
            g_bad.fetch_add(1);
          } else {
            tr.emplace_back(std::move(c.ctrl_sent.front()), std::vector<uint8_t>(f, f + hn + L));
            c.ctrl_sent.pop_front();
          }
        } else {
          if (f[0] != 0x81) g_bad.fetch_add(1);  // wsExample answers MessageText, FIN
          c.got.insert(c.got.end(), f + hn, f + hn + L);
        }
        off += hn + L;
      }
      c.in.erase(c.in.begin(), c.in.begin() + (long)off);
      if (c.state == 0 && c.ctrl_sent.empty() && c.got.size() >= c.data.size()) {
        if (c.got != c.data) g_bad.fetch_add(1);  // bytes.Equal (wsserver_test.go:128-130)
        c.done++;
        if (now_s() >= t_end) {
          if (g_cfg.close_end) ws_client_close(c, rng);
        } else {
          ws_client_next(c, rng);
        }
      }
    }
  }
  uint64_t sum = 0;
  for (auto& c : cs) {
    sum += c.done;
    if (g_cfg.close_end && c.state != 2) g_bad.fetch_add(1);  // closing handshake unfinished
    close(c.fd);
  }
  total->fetch_add(sum);
  close(ep);
  std::lock_guard<std::mutex> g(g_tr_mu);
  for (auto& p : tr) g_transcript.push_back(std::move(p));
}

// ------------------------------------------------------------------ wsserver_test.go:135-178 client
// TestWebSocketServer_CloseConnection: n clients dial and upgrade (the server
// counts OnConnect), then to_close of them close -- x/net/websocket's
// Conn.Close writes a close frame and closes the socket (--close-frame 1), or a
// bare TCP close (0) -- and after the drain (the reference sleeps 3 s) the
// server's live count must be n - to_close.  Then the rest close and the count
// must drain to 0.  Returns the counts seen.
struct CloseResult {
  int64_t after_connect = -1, after_close = -1, at_end = -1;
  int upgraded = 0;
  double drain_s = 0;
};

inline int64_t wait_live(int64_t want, double limit_s) {
  const double t0 = now_s();
  while (g_live.load() != want && now_s() - t0 < limit_s) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  return g_live.load();
}

inline CloseResult close_client(int port, int n, unsigned seed) {
  CloseResult res;
  std::mt19937_64 rng(seed);
  const char req_fmt[] =
      "GET / HTTP/1.1\r\nHost: 127.0.0.1:%d\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
      "Sec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\nOrigin: ws://127.0.0.1\r\nSec-WebSocket-Version: 13\r\n\r\n";
  char req[512];
  const int rn = snprintf(req, sizeof(req), req_fmt, port);
  std::vector<int> fds;
  for (int i = 0; i < n; ++i) {  // websocket.Dial: connect, upgrade request, wait for the 101
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (fd < 0 || connect(fd, (sockaddr*)&a, sizeof(a))) {
      perror("ws_loopback: connect");
      _exit(2);
    }
    fds.push_back(fd);
    send_all(fd, (const uint8_t*)req, (size_t)rn);
    std::string got;
    char b[1024];
    const double t0 = now_s();
    while (got.find("\r\n\r\n") == std::string::npos && now_s() - t0 < 5.0) {
      const ssize_t k = ::recv(fd, b, sizeof(b), 0);
      if (k <= 0) break;
      got.append(b, (size_t)k);
    }
    if (got.compare(0, 12, "HTTP/1.1 101") == 0 && got.find("s3pPLMBiTxaQ9kYGzzhZRbK+xOo=") != std::string::npos)
      ++res.upgraded;
    else
      g_bad.fetch_add(1);
  }
  res.after_connect = wait_live(n, 3.0);  // assert.Equal(t, n, ClientNum)
  const double tc = now_s();
  for (int i = 0; i < g_cfg.to_close && i < n; ++i) {
    if (g_cfg.close_frame) {  // Conn.Close: WriteClose(1000), then rwc.Close
      const uint8_t body[2] = {0x03, 0xE8};
      auto f = masked_frame(rng, 0x88, body, 2);
      if (!send_all(fds[i], f.data(), f.size())) g_bad.fetch_add(1);
    }
    close(fds[i]);
  }
  res.after_close = wait_live(n - g_cfg.to_close, 3.0);  // time.Sleep(3 s); assert n - toClose
  res.drain_s = now_s() - tc;
  for (int i = g_cfg.to_close; i < n; ++i) close(fds[i]);
  res.at_end = wait_live(0, 3.0);
  return res;
}

// The batched passes' timeline per pass in microseconds (whole run, warm-up
// included): host select / stage / launch / wait / deliver, and for passes
// answered by the completion flag the kernels' own GPU time.
inline std::string timeline_json() {
  const gevws_protocol_timeline& t = g_tl;
  if (t.passes == 0) return "null";
  const double p = (double)t.passes, s = t.signalled ? (double)t.signalled : 1.0;
  char b[512];
  snprintf(b, sizeof(b),
           "{\"passes\": %llu, \"select\": %.2f, \"stage\": %.2f, \"launch\": %.2f, \"wait\": %.2f, "
           "\"deliver\": %.2f, \"signalled_share\": %.3f, \"gpu_decode\": %.2f, \"gpu_handler\": %.2f, "
           "\"gpu_gap\": %.2f, \"service_share\": %.3f, \"direct_share\": %.3f}",
           (unsigned long long)t.passes, t.ns_select / p / 1e3, t.ns_stage / p / 1e3, t.ns_launch / p / 1e3,
           t.ns_wait / p / 1e3, t.ns_deliver / p / 1e3, t.signalled / p, t.ns_gpu_decode / s / 1e3,
           t.ns_gpu_handler / s / 1e3, t.ns_gpu_gap / s / 1e3, g_service_passes.load() / p, g_direct_passes.load() / p);
  return b;
}

template <class Decoder>
int loopback_main(int argc, char** argv) {
  int conns = 1000, loops = 1, cthreads = 4, port = 0, device = 0, ndev = 1;
  size_t msg = 128;
  double seconds = 5.0;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i];
    const char* v = argv[i + 1];
    if (k == "--conns") conns = atoi(v);
    else if (k == "--msg") msg = (size_t)atol(v);
    else if (k == "--seconds") seconds = atof(v);
    else if (k == "--loops") loops = atoi(v);
    else if (k == "--client-threads") cthreads = atoi(v);
    else if (k == "--port") port = atoi(v);
    else if (k == "--device") device = atoi(v);
    else if (k == "--devices") ndev = atoi(v) > 0 ? atoi(v) : 1;
    else if (k == "--mode")
      g_cfg.mode = std::string(v) == "wsserver" ? kModeWsServer : std::string(v) == "close" ? kModeClose : kModeEcho;
    else if (k == "--to-close") g_cfg.to_close = atoi(v);
    else if (k == "--close-frame") g_cfg.close_frame = atoi(v) != 0;
    else if (k == "--ctrl") g_cfg.ctrl_prob = atof(v);
    else if (k == "--close-end") g_cfg.close_end = atoi(v) != 0;
    else if (k == "--transcript") g_cfg.transcript = v;
    else if (k == "--seed") g_cfg.seed = (unsigned)atoi(v);
  }
  const bool wss = g_cfg.mode == kModeWsServer;
  if (!Decoder::kHandler && (g_cfg.ctrl_prob > 0 || g_cfg.close_end || (g_cfg.mode == kModeClose && g_cfg.close_frame))) {
    fprintf(stderr, "ws_loopback: control frames need the device handler (%s has none)\n", Decoder::name());
    return 2;
  }
  if (port == 0) port = 20000 + (int)(getpid() % 20000);
  // both ends of every connection live in this process: 2 fds per connection
  rlimit rl{};
  getrlimit(RLIMIT_NOFILE, &rl);
  rl.rlim_cur = rl.rlim_max;
  setrlimit(RLIMIT_NOFILE, &rl);
  if ((uint64_t)conns * 2 + 64 > (uint64_t)rl.rlim_cur) {
    fprintf(stderr, "ws_loopback: %d connections need %d fds, RLIMIT_NOFILE is %llu\n", conns, conns * 2 + 64,
            (unsigned long long)rl.rlim_cur);
    return 2;
  }
  std::atomic<int> ready{0};
  std::vector<std::thread> servers;
  for (int l = 0; l < loops; ++l) servers.emplace_back(server_loop<Decoder>, port, device + l % ndev, &ready, l);
  while (ready.load() < loops) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  if (g_cfg.mode == kModeClose) {
    const CloseResult r = close_client(port, conns, 77u * g_cfg.seed);
    g_stop = true;
    for (auto& t : servers) t.join();
    printf("{\"mode\": \"close\", \"decoder\": \"%s\", \"connections\": %d, \"upgraded\": %d, \"loops\": %d, "
           "\"to_close\": %d, \"close_frame\": %d, \"live_after_connect\": %lld, \"live_after_close\": %lld, "
           "\"live_at_end\": %lld, \"drain_s\": %.3f, \"closes_answered\": %llu, \"errors\": %llu}\n",
           Decoder::name(), conns, r.upgraded, loops, g_cfg.to_close, g_cfg.close_frame ? 1 : 0,
           (long long)r.after_connect, (long long)r.after_close, (long long)r.at_end, r.drain_s,
           (unsigned long long)g_closed.load(), (unsigned long long)g_bad.load());
    const bool ok = g_bad.load() == 0 && r.upgraded == conns && r.after_connect == conns &&
                    r.after_close == conns - g_cfg.to_close && r.at_end == 0;
    return ok ? 0 : 1;
  }

  std::atomic<uint64_t> total{0};
  std::atomic<int> upgraded{0};
  const double warm = 1.0;
  const double t0 = now_s();
  const double t_end = t0 + warm + seconds;
  std::vector<std::thread> clients;
  for (int t = 0; t < cthreads; ++t) {
    const int n = conns / cthreads + (t < conns % cthreads ? 1 : 0);
    if (wss)
      clients.emplace_back(ws_client_thread, port, n, t_end, &total, &upgraded, 1234u * g_cfg.seed + t);
    else
      clients.emplace_back(client_thread, port, n, msg, t_end, &total, &upgraded, 1234u + t);
  }
  // measure the steady state: count frames echoed between warm-up end and t_end
  std::this_thread::sleep_for(std::chrono::duration<double>(warm));
  const uint64_t f0 = g_frames.load(), b0 = g_batches.load(), c0 = g_batch_conns.load(), d0 = g_dev_ns.load();
  const uint64_t p0 = g_payload.load();
  std::vector<uint64_t> lf0(kMaxLoops), lf1(kMaxLoops);
  for (int l = 0; l < kMaxLoops; ++l) lf0[l] = g_loop_frames[l].load();
  const double ts = now_s();
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  const double te = now_s();
  const uint64_t f1 = g_frames.load(), b1 = g_batches.load(), c1 = g_batch_conns.load(), d1 = g_dev_ns.load();
  const uint64_t p1 = g_payload.load();
  for (int l = 0; l < kMaxLoops; ++l) lf1[l] = g_loop_frames[l].load();
  for (auto& t : clients) t.join();
  g_stop = true;
  for (auto& t : servers) t.join();
  const double dt = te - ts;
  const double mps = (double)(f1 - f0) / dt;
  // per-loop echo rates and connection counts (loops beyond kMaxLoops share
  // slots); fairness = min / max over loops of the echo rate per connection
  std::string per_loop = "[", per_conns = "[";
  double lmin = 0, lmax = 0;
  for (int l = 0; l < std::min(loops, kMaxLoops); ++l) {
    const double r = (double)(lf1[l] - lf0[l]) / dt;
    const uint64_t nc = g_loop_conns[l].load();
    const double rc = nc ? r / (double)nc : 0.0;
    lmin = l == 0 ? rc : std::min(lmin, rc);
    lmax = l == 0 ? rc : std::max(lmax, rc);
    char b[64];
    snprintf(b, sizeof(b), "%s%.0f", l ? ", " : "", r);
    per_loop += b;
    snprintf(b, sizeof(b), "%s%llu", l ? ", " : "", (unsigned long long)nc);
    per_conns += b;
  }
  per_loop += "]";
  per_conns += "]";
  if (!g_cfg.transcript.empty()) {
    FILE* tf = fopen(g_cfg.transcript.c_str(), "w");
    if (!tf) {
      perror("ws_loopback: transcript");
      return 2;
    }
    for (auto& p : g_transcript) {
      for (uint8_t b : p.first) fprintf(tf, "%02x", b);
      fputc(' ', tf);
      for (uint8_t b : p.second) fprintf(tf, "%02x", b);
      fputc('\n', tf);
    }
    fclose(tf);
  }
  printf("{\"path\": \"loopback websocket echo server: epoll loops -> ring buffers -> %s -> echo\", "
         "\"decoder\": \"%s\", \"connections\": %d, \"upgraded\": %d, "
         "\"msg_bytes\": %zu, \"loops\": %d, \"client_threads\": %d, \"seconds\": %.3f, "
         "\"echoes_per_s\": %.1f, \"payload_MiBps_each_way\": %.2f, \"decode_passes_per_s\": %.1f, "
         "\"mean_conns_per_pass\": %.1f, \"decode_us_per_pass\": %.1f, \"decode_share_of_loop_time\": %.3f, "
         "\"client_checked_echoes\": %llu, \"mode\": \"%s\", \"control_frames\": %llu, "
         "\"async_sends\": %llu, \"closes_answered\": %llu, \"transcript_pairs\": %zu, \"devices\": %d, "
         "\"pass_timeline_us\": %s, \"loop_echoes_per_s\": %s, \"loop_conns\": %s, "
         "\"loop_min_over_max_per_conn\": %.3f, "
         "\"errors\": %llu}\n",
         Decoder::path(), Decoder::name(), conns, upgraded.load(), wss ? (size_t)0 : msg, loops, cthreads, dt, mps,
         (double)(p1 - p0) / dt / 1048576.0, (double)(b1 - b0) / dt,
         b1 > b0 ? (double)(c1 - c0) / (double)(b1 - b0) : 0.0,
         b1 > b0 ? (double)(d1 - d0) / 1e3 / (double)(b1 - b0) : 0.0, (double)(d1 - d0) / 1e9 / (dt * loops),
         (unsigned long long)total.load(), wss ? "wsserver" : "echo", (unsigned long long)g_ctrl.load(),
         (unsigned long long)g_sent_async.load(), (unsigned long long)g_closed.load(), g_transcript.size(), ndev,
         timeline_json().c_str(), per_loop.c_str(), per_conns.c_str(), lmax > 0 ? lmin / lmax : 0.0, (unsigned long long)g_bad.load());
  return g_bad.load() == 0 && upgraded.load() == conns ? 0 : 1;
}

}  // namespace wslb

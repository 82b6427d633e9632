# Builds the product library (HIP, gfx950) and the test-only oracle.
#   make            -> pollnet_amd/libpollnet_amd.so + oracle/liboracle.so (+ oracle/_ref when /root/reference exists)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
CFLAGS_ORACLE = -O3 -march=x86-64-v3 -fPIC -Wall -std=c11

LIB = pollnet_amd/libpollnet_amd.so
SRCS = pollnet_amd/csrc/rx_kernel.hip pollnet_amd/csrc/rx_service.hip pollnet_amd/csrc/stream_kernel.hip pollnet_amd/csrc/tx_kernel.hip \
  pollnet_amd/csrc/conn_table.cpp
# the seeded workload generator (tests, bench): its own library, outside the product ABI
GEN_LIB = pollnet_amd/libpollnet_amd_gen.so
HDRS = include/pollnet_amd.h
KHDRS = pollnet_amd/csrc/frame_pass.hpp pollnet_amd/csrc/device_common.hpp pollnet_amd/csrc/pn_internal.hpp \
  pollnet_amd/csrc/rx_classify.hpp pollnet_amd/csrc/tx_fill.hpp pollnet_amd/csrc/stream_match.hpp
# measurement-only library (bench ceilings; A/B variants with TUNING=1): never loaded by the product
TUNING_LIB = pollnet_amd/libpollnet_amd_tuning.so
TUNING_SRCS = pollnet_amd/csrc/rx_tuning.hip pollnet_amd/csrc/tx_tuning.hip
TUNING ?= 1
ifeq ($(TUNING),1)
TUNING_FLAGS = -DPN_TUNING_VARIANTS
endif

ORACLE = oracle/liboracle.so
REFDIR ?= /root/reference

CPPTEST = tests/cpp/test_gpu_rx
RXCONNTEST = tests/cpp/test_rx_conn
TCPRXTEST = tests/cpp/test_gpu_tcp_rx
TCPRXBENCH = bench/bench_tcp_rx
LATBENCH = bench/bench_latency
SRVBENCH = bench/bench_tcp_server
PINBENCH = bench/bench_pinned
TXSMALLBENCH = bench/bench_tx_small
# (defined before `all`: make expands a rule's prerequisites where the rule is read)
SIGBENCH = bench/bench_signal
STREAMBENCH = bench/bench_streams
DOORBENCH = bench/bench_doorbell
RINGTEST = tests/cpp/test_rx_ring
STREAMTEST = tests/cpp/test_tcp_stream
GPUSTREAMTEST = tests/cpp/test_gpu_tcp_stream
SERVERTEST = tests/cpp/test_tcp_server
PEERTEST = tests/cpp/test_tcp_server_peer
CLISRVTEST = tests/cpp/test_tcp_client_server
TXHOSTTEST = tests/cpp/test_tx_host
REFSERVERTEST = tests/cpp/test_ref_server
REFCONNTEST = tests/cpp/test_ref_conn
REFCLIENTTEST = tests/cpp/test_ref_client

# Host programs that include HIP headers: compiled by hipcc with the device pass pinned to gfx950
# (without --offload-arch hipcc would add a default-arch device pass for nothing)
HOSTHIP = $(HIPCC) --offload-arch=$(ARCH)

# The two example-handler tests compile text the ref recipe extracts from /root/reference
# (oracle/_ref/*.inc, never committed, never sent to the GPU box).  Where neither that text nor
# the reference is present (a fresh GPU box), they are not rebuilt: their prebuilt binaries are used.
REF_INCS = oracle/_ref/tcpserver_handler.inc oracle/_ref/tcpclient_handler.inc
# efvitcp's own TcpConn / TcpServer / EfviTcpServer and Core's ef_vi-free members (oracle/ref.mk `conn`)
CONN_INCS = $(addprefix oracle/_ref/,conn_tcpconn.inc conn_tcpserver.inc conn_efvitcpserver.inc conn_timer_types.inc \
  conn_sendbuf.inc conn_core_consts.inc conn_core_init.inc conn_core_getns.inc conn_core_rst.inc conn_core_rx.inc \
  conn_core_tbl.inc conn_core_timer.inc conn_core_members.inc core_defs.inc conn_tcpclient_head.inc \
  conn_tcpclient_tail.inc conn_efvitcpclient.inc conn_core_autoport.inc)
HAVE_REF_TEXT = $(or $(wildcard $(REFDIR)/example/tcpserver.cc),$(and $(wildcard oracle/_ref/tcpserver_handler.inc),$(wildcard oracle/_ref/tcpclient_handler.inc)))
REF_TESTS = $(if $(HAVE_REF_TEXT),$(SERVERTEST) $(CLISRVTEST) $(REFSERVERTEST) $(REFCONNTEST) $(REFCLIENTTEST))

all: $(LIB) $(GEN_LIB) $(TUNING_LIB) $(ORACLE) ref $(CPPTEST) $(RXCONNTEST) $(TCPRXTEST) $(TCPRXBENCH) $(LATBENCH) $(SRVBENCH) $(PINBENCH) $(SIGBENCH) $(STREAMBENCH) $(DOORBENCH) $(RINGTEST) $(STREAMTEST) $(GPUSTREAMTEST) $(REF_TESTS) $(PEERTEST) $(TXHOSTTEST)

# GpuTcpServer (pollnet's EfviTcpServer surface) running the reference example's own handler
# (oracle/_ref/tcpserver_handler.inc, extracted by oracle/ref.mk) on the GPU vs a sequential twin
$(SERVERTEST): tests/cpp/test_tcp_server.cpp tests/cpp/segframes.hpp tests/cpp/server_harness.hpp include/pollnet_amd/tcp_server.hpp include/pollnet_amd/tcp_engine.hpp \
  include/pollnet_amd/rx_conn.hpp include/pollnet_amd/gpu_rx.hpp include/pollnet_amd/rx_ring.hpp $(HDRS) $(LIB) $(ORACLE) \
  oracle/_ref/tcpserver_handler.inc
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

$(REF_INCS) $(CONN_INCS):
	@if [ -d $(REFDIR) ]; then $(MAKE) -C oracle -f ref.mk REFDIR=$(REFDIR) $(@:oracle/%=%); \
	else echo "$@: no $(REFDIR) to extract it from" >&2; exit 1; fi

# GpuTcpServer (twin and GPU) vs the reference's own EfviTcpServer / TcpServer / TcpConn (oracle/ref_server.hpp)
$(REFSERVERTEST): tests/cpp/test_ref_server.cpp tests/cpp/peer_population.hpp tests/cpp/segframes.hpp tests/cpp/server_harness.hpp \
  oracle/ref_server.hpp include/pollnet_amd/tcp_server.hpp include/pollnet_amd/tcp_engine.hpp include/pollnet_amd/rx_conn.hpp \
  include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE) $(CONN_INCS)
	$(HOSTHIP) -O2 -std=c++17 -Wall -Wno-unused-result -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# GpuTcpClient (twin and GPU) vs the reference's own EfviTcpClient / TcpClient against a scripted server
$(REFCLIENTTEST): tests/cpp/test_ref_client.cpp tests/cpp/segframes.hpp tests/cpp/server_harness.hpp oracle/ref_server.hpp \
  include/pollnet_amd/tcp_client.hpp include/pollnet_amd/tcp_engine.hpp include/pollnet_amd/rx_conn.hpp \
  include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE) $(CONN_INCS)
	$(HOSTHIP) -O2 -std=c++17 -Wall -Wno-unused-result -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# RxConn (the receive half) vs the reference's own TcpConn::onPack, segment by segment (host only)
$(REFCONNTEST): tests/cpp/test_ref_conn.cpp tests/cpp/segframes.hpp oracle/ref_server.hpp include/pollnet_amd/rx_conn.hpp \
  $(HDRS) $(ORACLE) $(CONN_INCS)
	g++ -O2 -std=c++17 -Wall -Wno-unused-result -o $@ $< -Loracle -loracle -Wl,-rpath,'$$ORIGIN/../../oracle'

# GpuTcpClient <-> GpuTcpServer running both reference example handlers over a lossy in-memory wire
$(CLISRVTEST): tests/cpp/test_tcp_client_server.cpp tests/cpp/segframes.hpp tests/cpp/server_harness.hpp oracle/ref_server.hpp $(CONN_INCS) \
  include/pollnet_amd/tcp_client.hpp include/pollnet_amd/tcp_server.hpp include/pollnet_amd/tcp_engine.hpp \
  include/pollnet_amd/rx_conn.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE) \
  oracle/_ref/tcpserver_handler.inc oracle/_ref/tcpclient_handler.inc
	$(HOSTHIP) -O2 -std=c++17 -Wall -Wno-unused-function -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# GpuTcpServer against reactive in-memory TCP peers (loss, timers, windows), GPU vs twin
$(PEERTEST): tests/cpp/test_tcp_server_peer.cpp tests/cpp/segframes.hpp tests/cpp/server_harness.hpp tests/cpp/peer_population.hpp \
  include/pollnet_amd/tcp_server.hpp include/pollnet_amd/tcp_engine.hpp include/pollnet_amd/rx_conn.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# TcpStream reassembly restated vs the reference's own TcpStream (4 instantiations)
$(STREAMTEST): tests/cpp/test_tcp_stream.cpp tests/cpp/segframes.hpp include/pollnet_amd/tcp_stream.hpp $(HDRS) $(LIB) $(ORACLE)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle -ldl \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# pn_match_streams + GpuTcpStreams vs the reference filterPacket / TcpStream (GPU)
$(GPUSTREAMTEST): tests/cpp/test_gpu_tcp_stream.cpp tests/cpp/segframes.hpp include/pollnet_amd/tcp_stream.hpp \
  include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle -ldl \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# RX-ring ingestion: socket batcher (+ loopback capture when permitted), ef_vi event rings on the GPU
$(RINGTEST): tests/cpp/test_rx_ring.cpp include/pollnet_amd/rx_ring.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE) $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_gen -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# batch size vs throughput and latency of pn_classify (resident, host ring in/records out, hipGraph)
$(LATBENCH): bench/bench_latency.cpp $(HDRS) $(LIB) $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_gen -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# poll() throughput (GPU-classified) vs the same host loop over the CPU release path
$(TCPRXBENCH): bench/bench_tcp_rx.cpp tests/cpp/segframes.hpp include/pollnet_amd/gpu_tcp_rx.hpp \
  include/pollnet_amd/rx_conn.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE)
	$(HOSTHIP) -O3 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../oracle'

# GpuTcpServer::poll throughput (handshake, RX, ACKs) on the GPU vs the same server on the sequential backend
# (with the reference's own server as the release-path CPU leg where its text is present: oracle/ref_server.hpp)
$(SRVBENCH): bench/bench_tcp_server.cpp bench/sampler.hpp tests/cpp/segframes.hpp tests/cpp/server_harness.hpp include/pollnet_amd/tcp_server.hpp \
  include/pollnet_amd/tcp_engine.hpp include/pollnet_amd/rx_conn.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE) \
  $(if $(HAVE_REF_TEXT),oracle/ref_server.hpp $(CONN_INCS))
	$(HOSTHIP) -O3 -g -std=c++17 -Wall -Wno-unused-result -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../oracle'

# TX fill at small batch sizes, one in-place launch vs two phases (variant 41: make TUNING=1; not in `all`)
$(TXSMALLBENCH): bench/bench_tx_small.cpp $(HDRS) include/pollnet_amd_tuning.h $(LIB) $(TUNING_LIB) $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_gen -lpollnet_amd_tuning -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# completion by a polled word (pn_classify_notify) vs stream sync, small batches
$(SIGBENCH): bench/bench_signal.cpp $(HDRS) $(LIB) $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_gen -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# GPU round-trip latency floor: launch per request vs a resident kernel polling a doorbell (tuning library)
$(DOORBENCH): bench/bench_doorbell.cpp $(HDRS) include/pollnet_amd_tuning.h $(LIB) $(TUNING_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_tuning -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# the sniffer path end to end: GpuTcpStreams::poll vs every stream's filterPacket + handlePacket on one core
$(STREAMBENCH): bench/bench_streams.cpp include/pollnet_amd/tcp_stream.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB)
	$(HOSTHIP) -O3 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# zero-copy classify from host rings of each pinned-memory kind: PCIe rate and staleness
$(PINBENCH): bench/bench_pinned.cpp $(HDRS) $(LIB) $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_gen -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# receive-side server loop on the GPU vs a sequential twin with reference semantics
$(TCPRXTEST): tests/cpp/test_gpu_tcp_rx.cpp tests/cpp/segframes.hpp include/pollnet_amd/gpu_tcp_rx.hpp \
  include/pollnet_amd/rx_conn.hpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# the engine's host-side TX checksums vs the oracle's fill (host only)
$(TXHOSTTEST): tests/cpp/test_tx_host.cpp include/pollnet_amd/tcp_engine.hpp $(HDRS) $(LIB) $(ORACLE)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lpollnet_amd -lpollnet_amd -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# receive-side state machine (host only): scenarios + differential vs the reference TcpStream
$(RXCONNTEST): tests/cpp/test_rx_conn.cpp tests/cpp/segframes.hpp include/pollnet_amd/rx_conn.hpp $(HDRS) $(ORACLE)
	g++ -O2 -std=c++17 -Wall -o $@ $< -Loracle -loracle -ldl -Wl,-rpath,'$$ORIGIN/../../oracle'

# standalone C++ adapter test (no torch): links the product library and, as the checker, the oracle
$(CPPTEST): tests/cpp/test_gpu_rx.cpp include/pollnet_amd/gpu_rx.hpp $(HDRS) $(LIB) $(ORACLE) $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -o $@ $< -Lpollnet_amd -lpollnet_amd -lpollnet_amd_gen -Loracle -loracle \
	  -Wl,-rpath,'$$ORIGIN/../../pollnet_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

$(LIB): $(SRCS) $(HDRS) $(KHDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS) -lpthread

# the generator draws one RNG value per statement: any C++17 compiler gives the same frames
# (tests/test_build.py builds it with g++ and clang and checks the committed slices)
$(GEN_LIB): pollnet_amd/csrc/framegen.cpp include/pollnet_amd_gen.h $(HDRS) $(LIB)
	g++ -O3 -std=c++17 -fPIC -Wall -shared -o $@ pollnet_amd/csrc/framegen.cpp -Lpollnet_amd -lpollnet_amd -lpthread \
	  -Wl,-rpath,'$$ORIGIN'

$(TUNING_LIB): $(TUNING_SRCS) $(HDRS) include/pollnet_amd_tuning.h $(KHDRS)
	$(HIPCC) $(HIPFLAGS) $(TUNING_FLAGS) -shared -o $@ $(TUNING_SRCS)

$(ORACLE): oracle/pn_oracle.c oracle/pn_tx_oracle.c oracle/pn_oracle.h $(HDRS)
	gcc $(CFLAGS_ORACLE) -shared -o $@ oracle/pn_oracle.c oracle/pn_tx_oracle.c -lpthread

ref:
	@if [ -d $(REFDIR) ]; then $(MAKE) -C oracle -f ref.mk REFDIR=$(REFDIR); else echo "no $(REFDIR): using prebuilt oracle/_ref"; fi

clean:
	rm -f $(LIB) $(GEN_LIB) $(TUNING_LIB) $(ORACLE) oracle/_ref/*.so $(CPPTEST) $(RXCONNTEST) $(TCPRXTEST) $(TCPRXBENCH) $(LATBENCH) $(SRVBENCH) $(PINBENCH) $(SIGBENCH) $(STREAMBENCH) $(DOORBENCH) $(TXSMALLBENCH) $(RINGTEST) $(STREAMTEST) $(GPUSTREAMTEST) $(SERVERTEST) $(PEERTEST) $(CLISRVTEST) $(TXHOSTTEST) $(REFSERVERTEST) $(REFCONNTEST) $(REFCLIENTTEST)

.PHONY: all ref clean svc_trace

# Measurement build of the service with its step clocks (-DPN_SVC_TRACE) and the driver that reads them; not in `all`
svc_trace: ab_libs/trace/libpollnet_amd.so bench/svc_trace
ab_libs/trace/libpollnet_amd.so: $(SRCS) $(HDRS) $(KHDRS)
	mkdir -p ab_libs/trace
	$(HIPCC) $(HIPFLAGS) -DPN_SVC_TRACE -shared -o $@ $(SRCS) -lpthread
bench/svc_trace: bench/svc_trace.cpp ab_libs/trace/libpollnet_amd.so $(GEN_LIB)
	$(HOSTHIP) -O2 -std=c++17 -Wall -o $@ $< -Lab_libs/trace -lpollnet_amd -Lpollnet_amd -lpollnet_amd_gen \
	  -Wl,-rpath,'$$ORIGIN/../ab_libs/trace' -Wl,-rpath,'$$ORIGIN/../pollnet_amd'

# Builds oracle/_ref from the reference's own sources where they lie (read-only).
# Buildable here: TcpStream.h (header-only), Socket.h (BSD sockets, config C1), and the
# hot-path parts of efvitcp/Core.h that touch no ef_vi type (line ranges below).  The whole
# Core.h needs <etherfabric/*.h> (ef_vi, not installed); stand-ins for those headers are not
# allowed, so Core.h as a unit is not built.
REFDIR ?= /root/reference
all: conn _ref/libref_tcpstream.so _ref/ref_socket_c1 _ref/tcpserver_handler.inc _ref/tcpclient_handler.inc _ref/libref_core.so

_ref/libref_tcpstream.so: ref_tcpstream.cc $(REFDIR)/TcpStream.h
	mkdir -p _ref
	g++ -O2 -std=c++17 -fPIC -shared -I$(REFDIR) -o $@ ref_tcpstream.cc

# BASELINE C1: the reference's Socket.h server + client, 1500-B echo over loopback
_ref/ref_socket_c1: ref_socket_c1.cc $(REFDIR)/Socket.h
	mkdir -p _ref
	g++ -O3 -std=c++17 -Wall -pthread -I$(REFDIR) -o $@ ref_socket_c1.cc

.PHONY: all

# The handler of the reference's example server (example/tcpserver.cc:61-90, the
# `struct { ... } handler;` the example polls with), extracted verbatim so that
# tests/cpp/test_tcp_server.cpp compiles it unchanged against GpuTcpServer.  Generated
# into _ref/ (git-ignored); the test binary built from it travels, the text does not.
_ref/tcpserver_handler.inc: $(REFDIR)/example/tcpserver.cc
	mkdir -p _ref
	sed -n '61,90p' $< > $@
	grep -q 'onTcpData' $@ && grep -q '} handler;' $@

# The handler of the reference's example client (example/tcpclient.cc:68-95), the same way.
_ref/tcpclient_handler.inc: $(REFDIR)/example/tcpclient.cc
	mkdir -p _ref
	sed -n '68p' $< | grep -q struct && sed -n '70p' $< | grep -q onTcpConnectFailed && sed -n '95p' $< | grep -q '} handler;'
	sed -n '68,95p' $< > $@

# The reference's own Core.h code for the hot path (CSum, headers, connHashKey, the conn
# table's member functions, Core::checksum), extracted verbatim by line range and compiled
# inside the harness class of ref_core.cc.  Each range is checked to start and end where
# expected, so a changed reference fails the build instead of compiling the wrong lines.
CORE = $(REFDIR)/efvitcp/Core.h
_ref/core_defs.inc: $(CORE)
	mkdir -p _ref
	sed -n '44p' $< | grep -q 'RecvMSS' && sed -n '138p' $< | grep -q '^};' && sed -n '167p' $< | grep -q 'connHashKey' && sed -n '182p' $< | grep -q '^};'
	sed -n '44,138p;167,182p' $< > $@
_ref/core_sizes.inc: $(CORE)
	mkdir -p _ref
	sed -n '235p' $< | grep -q MaxTableSize && sed -n '236p' $< | grep -q TotalTableSize
	sed -n '235,236p' $< > $@
_ref/core_table.inc: $(CORE)
	mkdir -p _ref
	sed -n '558p' $< | grep -q findConnEntry && sed -n '605p' $< | grep -q '^  }' && sed -n '640p' $< | grep -q EFVITCP_DEBUG && sed -n '650p' $< | grep -q tryExpandConnTbl && sed -n '682p' $< | grep -q '^  }'
	sed -n '558,605p;640,648p;650,682p' $< > $@
_ref/core_checksum.inc: $(CORE)
	mkdir -p _ref
	sed -n '448p' $< | grep -q EFVITCP_DEBUG && sed -n '449p' $< | grep -q 'void checksum' && sed -n '472p' $< | grep -q endif
	sed -n '448,472p' $< > $@
# TcpConn::onPack's first statements (TcpConn.h:469-473): payload start/end and seq + syn
_ref/onpack_head.inc: $(REFDIR)/efvitcp/TcpConn.h
	mkdir -p _ref
	sed -n '468p' $< | grep -q 'void onPack' && sed -n '473p' $< | grep -q 'seq_num' && sed -n '474p' $< | grep -q got_ts
	sed -n '469,473p' $< > $@
# The send path's byte work (TX checksum fill parity): TcpConn::copyAndSum (TcpConn.h:257-299)
# and SendBuf::setOptDataLen (Core.h:157-163)
_ref/tx_copyandsum.inc: $(REFDIR)/efvitcp/TcpConn.h
	mkdir -p _ref
	sed -n '257p' $< | grep -q 'CSum copyAndSum' && sed -n '299p' $< | grep -q '^  }$$' && sed -n '300p' $< | grep -q '^$$'
	sed -n '257,299p' $< > $@
_ref/tx_setoptdatalen.inc: $(CORE)
	mkdir -p _ref
	sed -n '157p' $< | grep -q 'void setOptDataLen' && sed -n '163p' $< | grep -q '^  }$$'
	sed -n '157,163p' $< > $@
# Efvi's UDP send path (the PN_TX_UDP_EFVI contract): its header structs (Efvi.h:557-586, up to
# the ef_addr-holding pkt_buf), the cached IPv4 header sum (:406-411) and update_udp_pkt (:611-621)
EFVI = $(REFDIR)/Efvi.h
_ref/efvi_hdrs.inc: $(EFVI)
	mkdir -p _ref
	sed -n '557p' $< | grep -q 'pragma pack(push, 1)' && sed -n '558p' $< | grep -q ci_ether_hdr && sed -n '580p' $< | grep -q ci_udp_hdr && sed -n '586p' $< | grep -q '^  };$$'
	sed -n '557,586p' $< > $@
_ref/efvi_ipsum_cache.inc: $(EFVI)
	mkdir -p _ref
	sed -n '405p' $< | grep -q 'uint16_t\* ip4' && sed -n '406p' $< | grep -q 'ipsum_cache = 0;' && sed -n '411p' $< | grep -q 'ipsum_cache += (ipsum_cache >> 16u);'
	sed -n '406,411p' $< > $@
_ref/efvi_update_udp_pkt.inc: $(EFVI)
	mkdir -p _ref
	sed -n '611p' $< | grep -q 'void update_udp_pkt' && sed -n '621p' $< | grep -q '^  }$$'
	sed -n '611,621p' $< > $@
_ref/libref_core.so: ref_core.cc _ref/core_defs.inc _ref/core_sizes.inc _ref/core_table.inc _ref/core_checksum.inc _ref/onpack_head.inc \
  _ref/tx_copyandsum.inc _ref/tx_setoptdatalen.inc _ref/efvi_hdrs.inc _ref/efvi_ipsum_cache.inc _ref/efvi_update_udp_pkt.inc
	g++ -O3 -march=x86-64-v3 -std=c++17 -fPIC -shared -pthread -Wno-unused-result -o $@ ref_core.cc

# ---- efvitcp's whole receive/send state machine, for the F1 differential (tests/cpp/test_ref_conn.cpp,
# tests/cpp/test_ref_server.cpp).  TcpConn (TcpConn.h:29-914), TcpServer (TcpServer.h:29-121) and
# pollnet's EfviTcpServer wrapper (EfviTcp.h:188-313) are extracted whole; from Core.h every member
# that touches no ef_vi type (below), pasted into oracle/ref_server.hpp's harness Core, which
# restates only the ef_vi lines (init's driver/NIC calls, send's transmit, pollNet's event loop).
TCPCONN = $(REFDIR)/efvitcp/TcpConn.h
TCPSERVER = $(REFDIR)/efvitcp/TcpServer.h
EFVITCP = $(REFDIR)/efvitcp/EfviTcp.h
CONN_INCS = _ref/conn_tcpconn.inc _ref/conn_tcpserver.inc _ref/conn_efvitcpserver.inc _ref/conn_timer_types.inc \
  _ref/conn_sendbuf.inc _ref/conn_core_consts.inc _ref/conn_core_init.inc _ref/conn_core_getns.inc _ref/conn_core_rst.inc \
  _ref/conn_core_rx.inc _ref/conn_core_tbl.inc _ref/conn_core_timer.inc _ref/conn_core_members.inc
conn: $(CONN_INCS)
_ref/conn_tcpconn.inc: $(TCPCONN)
	mkdir -p _ref
	sed -n '29p' $< | grep -q '^template<typename Conf>$$' && sed -n '30p' $< | grep -q '^class TcpConn ' && sed -n '914p' $< | grep -q '^};$$' && sed -n '916p' $< | grep -q 'namespace efvitcp'
	sed -n '29,914p' $< > $@
_ref/conn_tcpserver.inc: $(TCPSERVER)
	mkdir -p _ref
	sed -n '29p' $< | grep -q '^template<typename Conf>$$' && sed -n '30p' $< | grep -q '^class TcpServer$$' && sed -n '121p' $< | grep -q '^};$$'
	sed -n '29,121p' $< > $@
_ref/conn_efvitcpserver.inc: $(EFVITCP)
	mkdir -p _ref
	sed -n '188p' $< | grep -q '^template<typename Conf>$$' && sed -n '189p' $< | grep -q '^class EfviTcpServer$$' && sed -n '313p' $< | grep -q '^};$$'
	sed -n '188,313p' $< > $@
# TimerNode, TimeWaitConn
_ref/conn_timer_types.inc: $(CORE)
	mkdir -p _ref
	sed -n '184p' $< | grep -q '^struct TimerNode$$' && sed -n '203p' $< | grep -q '^struct TimeWaitConn$$' && sed -n '214p' $< | grep -q '^};$$'
	sed -n '184,214p' $< > $@
# SendBuf's members after its ef_addr (send_ts .. setOptDataLen)
_ref/conn_sendbuf.inc: $(CORE)
	mkdir -p _ref
	sed -n '149p' $< | grep -q 'ef_addr post_addr' && sed -n '150p' $< | grep -q 'uint32_t send_ts;' && sed -n '163p' $< | grep -q '^  }$$' && sed -n '164p' $< | grep -q '^};$$'
	sed -n '150,163p' $< > $@
_ref/conn_core_consts.inc: $(CORE)
	mkdir -p _ref
	sed -n '232p' $< | grep -q SendBufSize && sed -n '236p' $< | grep -q TotalTableSize
	sed -n '232,236p' $< > $@
# Core::init after the ef_vi calls: send buffers (less their DMA address, :292), RST sums, id stacks, table
_ref/conn_core_init.inc: $(CORE)
	mkdir -p _ref
	sed -n '290p' $< | grep -q 'i < SendBufCnt' && sed -n '292p' $< | grep -q ef_memreg_dma_addr && sed -n '293p' $< | grep -q 'avail = true' && sed -n '322p' $< | grep -q 'tbl_mask = ' && sed -n '324p' $< | grep -q 'return nullptr'
	sed -n '290,291p;293,322p' $< > $@
_ref/conn_core_getns.inc: $(CORE)
	mkdir -p _ref
	sed -n '327p' $< | grep -q 'int64_t getns()' && sed -n '331p' $< | grep -q '^  }$$'
	sed -n '327,331p' $< > $@
# sumRst, rspRst, ackTW
_ref/conn_core_rst.inc: $(CORE)
	mkdir -p _ref
	sed -n '385p' $< | grep -q 'void sumRst' && sed -n '400p' $< | grep -q 'void rspRst' && sed -n '425p' $< | grep -q 'void ackTW' && sed -n '446p' $< | grep -q '^  }$$'
	sed -n '385,446p' $< > $@
# pollNet's RX-event body, after the event's request id (:503) and before the re-post (:529)
_ref/conn_core_rx.inc: $(CORE)
	mkdir -p _ref
	sed -n '503p' $< | grep -q EF_EVENT_RX_RQ_ID && sed -n '504p' $< | grep -q 'RecvBuf\* buf' && sed -n '526p' $< | grep -q 'recv_handler(key, entry, eth_hdr)' && sed -n '527p' $< | grep -q '^          }$$' && sed -n '529p' $< | grep -q ef_vi_receive_init
	sed -n '504,527p' $< > $@
# getSendBuf, findConnEntry .. tryExpandConnTbl (enterTW included)
_ref/conn_core_tbl.inc: $(CORE)
	mkdir -p _ref
	sed -n '554p' $< | grep -q 'SendBuf\* getSendBuf' && sed -n '607p' $< | grep -q 'void enterTW' && sed -n '682p' $< | grep -q '^  }$$'
	sed -n '554,682p' $< > $@
# addTimer, pollTime
_ref/conn_core_timer.inc: $(CORE)
	mkdir -p _ref
	sed -n '684p' $< | grep -q 'void addTimer' && sed -n '710p' $< | grep -q 'void pollTime' && sed -n '751p' $< | grep -q '^  }$$'
	sed -n '684,751p' $< > $@
# data members, less the ef_vi handles (:763-768)
_ref/conn_core_members.inc: $(CORE)
	mkdir -p _ref
	sed -n '753p' $< | grep -q SendBufCnt && sed -n '762p' $< | grep -q 'uint8_t\* pkt_buf;' && sed -n '763p' $< | grep -q 'ef_vi vi' && sed -n '768p' $< | grep -q use_ctpio && sed -n '769p' $< | grep -q 'local_mac' && sed -n '782p' $< | grep -q timer_slots && sed -n '783p' $< | grep -q '^};$$'
	sed -n '753,762p;769,782p' $< > $@
.PHONY: conn
# The client side: TcpClient (TcpClient.h:30-104 and 166-168; its getDestMac, :105-164, reads the
# host's route / ARP tables and is the harness's), pollnet's EfviTcpClient (EfviTcp.h:30-186) and
# Core::autoGetPort (Core.h:357-373)
TCPCLIENT = $(REFDIR)/efvitcp/TcpClient.h
CONN_INCS += _ref/conn_tcpclient_head.inc _ref/conn_tcpclient_tail.inc _ref/conn_efvitcpclient.inc _ref/conn_core_autoport.inc
conn: $(CONN_INCS)
_ref/conn_tcpclient_head.inc: $(TCPCLIENT)
	mkdir -p _ref
	sed -n '30p' $< | grep -q '^template<typename Conf>$$' && sed -n '31p' $< | grep -q '^class TcpClient$$' && sed -n '104p' $< | grep -q '^private:$$' && sed -n '105p' $< | grep -q getDestMac && sed -n '164p' $< | grep -q '^  }$$'
	sed -n '30,104p' $< > $@
_ref/conn_tcpclient_tail.inc: $(TCPCLIENT)
	mkdir -p _ref
	sed -n '166p' $< | grep -q 'Core<CliConf> core;' && sed -n '167p' $< | grep -q 'Conn conn;' && sed -n '168p' $< | grep -q '^};$$'
	sed -n '166,168p' $< > $@
_ref/conn_efvitcpclient.inc: $(EFVITCP)
	mkdir -p _ref
	sed -n '30p' $< | grep -q '^template<typename Conf>$$' && sed -n '31p' $< | grep -q '^class EfviTcpClient$$' && sed -n '186p' $< | grep -q '^};$$' && sed -n '188p' $< | grep -q '^template<typename Conf>$$'
	sed -n '30,186p' $< > $@
_ref/conn_core_autoport.inc: $(CORE)
	mkdir -p _ref
	sed -n '357p' $< | grep -q 'const char\* autoGetPort' && sed -n '373p' $< | grep -q '^  }$$'
	sed -n '357,373p' $< > $@

# Builds oracle/_ref from the reference's own sources where they lie (read-only).
# Buildable here: TcpStream.h (header-only), Socket.h (BSD sockets, config C1), and the
# hot-path parts of efvitcp/Core.h that touch no ef_vi type (line ranges below).  The whole
# Core.h needs <etherfabric/*.h> (ef_vi, not installed); stand-ins for those headers are not
# allowed, so Core.h as a unit is not built.
REFDIR ?= /root/reference
all: _ref/libref_tcpstream.so _ref/ref_socket_c1 _ref/tcpserver_handler.inc _ref/tcpclient_handler.inc _ref/libref_core.so

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

# Builds oracle/_ref from the reference's own sources where they lie (read-only).
# Buildable here: TcpStream.h (header-only) and Socket.h (BSD sockets, config C1).
# efvitcp/Core.h needs <etherfabric/*.h> (ef_vi, not installed) and stand-ins for those
# headers are not allowed, so it is not built.
REFDIR ?= /root/reference
all: _ref/libref_tcpstream.so _ref/ref_socket_c1 _ref/tcpserver_handler.inc

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

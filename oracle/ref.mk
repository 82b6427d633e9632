# Builds oracle/_ref from the reference's own sources where they lie (read-only).
# Buildable here: TcpStream.h (header-only) and Socket.h (BSD sockets, config C1).
# efvitcp/Core.h needs <etherfabric/*.h> (ef_vi, not installed) and stand-ins for those
# headers are not allowed, so it is not built.
REFDIR ?= /root/reference
all: _ref/libref_tcpstream.so _ref/ref_socket_c1

_ref/libref_tcpstream.so: ref_tcpstream.cc $(REFDIR)/TcpStream.h
	mkdir -p _ref
	g++ -O2 -std=c++17 -fPIC -shared -I$(REFDIR) -o $@ ref_tcpstream.cc

# BASELINE C1: the reference's Socket.h server + client, 1500-B echo over loopback
_ref/ref_socket_c1: ref_socket_c1.cc $(REFDIR)/Socket.h
	mkdir -p _ref
	g++ -O3 -std=c++17 -Wall -pthread -I$(REFDIR) -o $@ ref_socket_c1.cc

.PHONY: all

# Builds oracle/_ref from the reference's own sources where they lie (read-only).
# Only TcpStream.h is buildable here: efvitcp/Core.h needs <etherfabric/*.h>
# (ef_vi, not installed) and stand-ins for those headers are not allowed.
REFDIR ?= /root/reference
_ref/libref_tcpstream.so: ref_tcpstream.cc $(REFDIR)/TcpStream.h
	mkdir -p _ref
	g++ -O2 -std=c++17 -fPIC -shared -I$(REFDIR) -o $@ ref_tcpstream.cc

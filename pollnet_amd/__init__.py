"""pollnet_amd — MI355X-native receive-path per-frame transform for efvitcp.

Python host mirror over the C-ABI in ``include/pollnet_amd.h`` (libpollnet_amd.so,
built for gfx950).  The product path is the HIP kernel behind ``pn_classify``;
this module only marshals pointers.  There is no CPU fallback: if the shared
library is missing, importing the package raises.

Reference seam: efvitcp ``Core::pollNet`` (efvitcp/Core.h:494-552)
→ ``recv_handler(key, entry, eth)`` → ``TcpConn::onPack`` (efvitcp/TcpConn.h:469-473).
"""
from .rx import (  # noqa: F401
    LIB_PATH,
    PN_EMPTY_KEY,
    PN_MISS,
    PN_TX_TCP,
    PN_TX_UDP_EFVI,
    PN_TX_UDP,
    RESULT_DTYPE,
    ENTRY_DTYPE,
    STREAM_FILTER_DTYPE,
    PN_NO_STREAM,
    PN_MAX_STREAM_FILTERS,
    PN_SERVICE_WAVES,
    PN_SERVICE_WAVES_PER_CU,
    PN_SERVICE_MAX_WAVES,
    PN_SERVICE_MAX_FRAMES,
    PN_LINK_MAX_FRAMES,
    PN_LINK_MAX_CONNS,
    F,
    ConnTable,
    PollnetError,
    RxContext,
    RxService,
    conn_hash_key,
    device_count,
    gen_conn_table,
    gen_frames,
    wire_bytes,
)

"""Print the socket-API part of bench line(s): sequential, halves, overlapped
(unpinned / pinned) rates and where rx_burst's time went.
    python tools/sock_summary.py gpurun_out/bench.log"""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    for name, v in (d.get("socket_api") or {}).items():
        if "mpps" not in v:
            print(name, v)
            continue
        print(f"{name}: seq {v['mpps']} Mpps (rx {v['rx_burst_ms']} + app {v['app_recv_ms']} ms)")
        for k in ("halves", "ingest_pull", "overlapped", "overlapped_unpinned"):
            x = v.get(k)
            if not x:
                continue
            ph = x.get("rx_burst_phases_ms", {})
            print(f"  {k}: {x['mpps']} Mpps, rx {x['rx_burst_ms']} ms, app "
                  f"{x.get('app_drain_ms', x.get('app_recv_ms'))} ms, tcp_deliver "
                  f"{ph.get('tcp_deliver')}, udp_deliver {ph.get('udp_deliver')}, cpus {x.get('cpus')}, "
                  f"equal {x.get('received_equal')}, copied {x.get('copied_payload_bytes')}, "
                  f"waited {x.get('bursts_waited_for_buffer')}")
            if x.get("copied_mb_by_burst"):
                print("    copied MB by burst", x["copied_mb_by_burst"])
                print("    batches holding a buffer, by burst", x.get("held_batches_by_burst"))
                print("    app ms per burst", x.get("app_ms_per_burst"))

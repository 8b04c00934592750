# Network-policy probe: tries a TCP connection and reports the outcome.
import socket
import sys

host = sys.argv[1] if len(sys.argv) > 1 else "example.com"
try:
    with socket.create_connection((host, 80), timeout=3) as s:
        s.sendall(b"HEAD / HTTP/1.0\r\nHost: " + host.encode() + b"\r\n\r\n")
        print(s.recv(64))
except OSError as e:
    print("no egress:", e)

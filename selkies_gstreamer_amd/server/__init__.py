"""Streaming server (engine A of the reference: websocket data server, input, capture)."""

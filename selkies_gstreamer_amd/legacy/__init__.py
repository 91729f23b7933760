"""Legacy WebRTC-mode components (signalling server/client, RTC config)."""

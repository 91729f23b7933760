"""``selkies`` console script (reference src/selkies/__main__.py): the websocket
server, or ``selkies webrtc ...`` for the legacy WebRTC mode."""
import sys


def main() -> int:
    from selkies_gstreamer_amd.__main__ import _main
    return _main()


if __name__ == "__main__":
    sys.exit(main())

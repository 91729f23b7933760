"""``python -m selkies_gstreamer_amd`` == the ``selkies`` console script (reference __main__.py:14-16).

``python -m selkies_gstreamer_amd webrtc [flags]`` starts the legacy WebRTC mode
(reference legacy/webrtc.py main, which the reference ships without an entry point).
"""
import sys


def _main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "webrtc":
        from selkies_gstreamer_amd.legacy.webrtc_app import main as webrtc_main
        return webrtc_main(sys.argv[2:])
    from selkies_gstreamer_amd.server.app import main
    return main()


if __name__ == "__main__":
    sys.exit(_main())

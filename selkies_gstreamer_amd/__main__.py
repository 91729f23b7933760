"""``python -m selkies_gstreamer_amd`` == the ``selkies`` console script (reference __main__.py:14-16)."""
import sys

from selkies_gstreamer_amd.server.app import main

if __name__ == "__main__":
    sys.exit(main())

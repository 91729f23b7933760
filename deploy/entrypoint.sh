#!/bin/bash
# Starts the streaming server once the X server and audio are up
# (reference addons/example/selkies-gstreamer-entrypoint.sh, rewritten for the
# MI355X build: no GStreamer environment, no NVRTC download; the encoder is
# the in-tree HIP library).
set -e
export DISPLAY="${DISPLAY:-:20}"
export XDG_RUNTIME_DIR="${XDG_RUNTIME_DIR:-/tmp}"
export PULSE_RUNTIME_PATH="${PULSE_RUNTIME_PATH:-${XDG_RUNTIME_DIR}/pulse}"
export PULSE_SERVER="${PULSE_SERVER:-unix:${PULSE_RUNTIME_PATH}/native}"

# games see four virtual Xbox pads through the interposer + fake libudev
export SELKIES_INTERPOSER=/usr/lib/selkies_joystick_interposer.so
export SDL_JOYSTICK_DEVICE=/dev/input/js0

until [ -S "/tmp/.X11-unix/X${DISPLAY#*:}" ]; do sleep 0.5; done

# self-hosted TURN when nothing else is configured (the reference does the same)
if [ -z "${SELKIES_TURN_REST_URI}" ] && [ -z "${SELKIES_TURN_SHARED_SECRET}" ] && \
   { [ -z "${SELKIES_TURN_USERNAME}" ] || [ -z "${SELKIES_TURN_PASSWORD}" ]; }; then
  export SELKIES_TURN_HOST="${SELKIES_TURN_HOST:-$(hostname -I 2>/dev/null | awk '{print $1; exit}')}"
  export SELKIES_TURN_PORT="${SELKIES_TURN_PORT:-3478}"
  export SELKIES_TURN_USERNAME=selkies
  export SELKIES_TURN_PASSWORD="$(tr -dc 'A-Za-z0-9' < /dev/urandom | head -c 24)"
  export SELKIES_TURN_PROTOCOL="${SELKIES_TURN_PROTOCOL:-tcp}"
  /etc/start-turnserver.sh &
fi

cd /opt/selkies
if [ "${SELKIES_MODE:-websockets}" = "webrtc" ]; then
  exec python3 -m selkies_gstreamer_amd webrtc --addr=0.0.0.0 --port="${SELKIES_PORT}" "$@"
fi
exec python3 -m selkies_gstreamer_amd --port="${SELKIES_PORT}" "$@"

#!/bin/bash
# coturn with either the HMAC shared secret (time-limited credentials, what
# selkies' /turn endpoint and the TURN REST service hand out) or one long-term
# user (SELKIES_TURN_USERNAME / SELKIES_TURN_PASSWORD).
set -e
EXTERNAL_IP="${TURN_EXTERNAL_IP:-$(detect_external_ip.sh 2>/dev/null || true)}"
ARGS=(--verbose --listening-ip=0.0.0.0 --listening-port="${TURN_PORT:-${SELKIES_TURN_PORT:-3478}}"
      --realm="${TURN_REALM:-selkies}" --min-port="${TURN_MIN_PORT:-49152}" --max-port="${TURN_MAX_PORT:-65535}"
      --no-cli --fingerprint --no-multicast-peers --channel-lifetime=-1 --log-file=stdout)
[ -n "${EXTERNAL_IP}" ] && ARGS+=(--external-ip="${EXTERNAL_IP}")
SECRET="${TURN_SHARED_SECRET:-${SELKIES_TURN_SHARED_SECRET:-}}"
if [ -n "${SECRET}" ]; then
  ARGS+=(--use-auth-secret --static-auth-secret="${SECRET}")
else
  ARGS+=(--lt-cred-mech --user="${SELKIES_TURN_USERNAME:-selkies}:${SELKIES_TURN_PASSWORD:?set a TURN password}")
fi
[ "${TURN_PROMETHEUS:-false}" = "true" ] && ARGS+=(--prometheus)
exec turnserver "${ARGS[@]}"

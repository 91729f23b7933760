#!/bin/bash
# Prints this host's public IPv4 address (cloud metadata first, then DNS, then
# the first local address), used as coturn's --external-ip.
set -u
for url in "http://169.254.169.254/latest/meta-data/public-ipv4" \
           "http://metadata.google.internal/computeMetadata/v1/instance/network-interfaces/0/access-configs/0/external-ip"; do
  ip="$(curl -fs -m 2 -H 'Metadata-Flavor: Google' "$url" 2>/dev/null)" && [ -n "$ip" ] && { echo "$ip"; exit 0; }
done
ip="$(dig -4 TXT +short @ns1.google.com o-o.myaddr.l.google.com 2>/dev/null | tr -d '"')"
[ -n "$ip" ] && { echo "$ip"; exit 0; }
hostname -I 2>/dev/null | awk '{print $1; exit}'

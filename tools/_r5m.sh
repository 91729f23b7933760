A="--encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu_steps.sh "pmc r5m_av1pmc $A" "prof r5m_av1prof $A" "driver r5m_driver"

package config

// Node configuration of the GPU signature verifier (SURVEY.md §5): app.toml
// keys under [gpu-verify], next to the BaseConfig of server/config/config.go.
//
// Patch (two lines): add the field to Config (config.go:44-47)
//
//	GPUVerify GPUVerifyConfig `mapstructure:"gpu-verify"`
//
// and DefaultGPUVerifyConfig() to DefaultConfig (config.go:78-88); append
// GPUVerifyTemplate to the app.toml template (server/config/toml.go).  The
// start command binds the matching flags (server/gpuverify_flags.go).

import (
	"fmt"
	"strconv"
	"strings"
	"time"
)

// GPUVerifyConfig: every knob of the verifier a node operator sets.
type GPUVerifyConfig struct {
	// Enable routes signature checks to the GPU; false keeps the reference
	// CPU path (the decorator then verifies with gpuverify.CPU).
	Enable bool `mapstructure:"enable"`
	// Devices: comma-separated HIP device ids ("" = every visible device).
	Devices string `mapstructure:"devices"`
	// MaxBatch: largest batch one device call takes (gv_set_option max_batch).
	MaxBatch int `mapstructure:"max-batch"`
	// CPUBelow: batches with fewer leaves run the reference VerifyBytes.
	CPUBelow int `mapstructure:"cpu-below"`
	// Keyed: verify through the HBM account-key arena (SURVEY.md §8f-2).
	Keyed bool `mapstructure:"keyed"`
	// KeyLoadMin: smallest batch that loads keys into the arena.
	KeyLoadMin int `mapstructure:"key-load-min"`
	// KeyCap, EdKeyCap: arena sizes at which the arenas are reset.
	KeyCap   int `mapstructure:"key-cap"`
	EdKeyCap int `mapstructure:"ed-key-cap"`
	// CacheEntries: the verdict cache (0 = no cache).
	CacheEntries int `mapstructure:"cache-entries"`
	// CheckTxWindowTxs / CheckTxWindow: the concurrent-CheckTx accumulation
	// window (baseapp.CheckTxWindow; a lone request never waits).
	CheckTxWindowTxs int           `mapstructure:"checktx-window-txs"`
	CheckTxWindow    time.Duration `mapstructure:"checktx-window"`
	// PreVerifyBlocks: pre-verify each block before its DeliverTx loop
	// (baseapp.PreVerifyTxs) and, where blocks are known ahead, the next one
	// beside it (PreVerifyAhead).
	PreVerifyBlocks bool `mapstructure:"preverify-blocks"`
}

// DefaultGPUVerifyConfig: off by default (a node opts in), the library's own
// defaults otherwise (include/gpuverify.h: GV_CPU_CROSSOVER, GV_KEY_LOAD_MIN,
// GV_KEY_CAP, GV_ED_KEY_CAP; the CheckTx window of the C++ mirror).
func DefaultGPUVerifyConfig() GPUVerifyConfig {
	return GPUVerifyConfig{
		Enable: false, Devices: "", MaxBatch: 1 << 20, CPUBelow: 4, Keyed: true, KeyLoadMin: 4096,
		KeyCap: 1 << 22, EdKeyCap: 1 << 16, CacheEntries: 1 << 20, CheckTxWindowTxs: 64,
		CheckTxWindow: 200 * time.Microsecond, PreVerifyBlocks: true,
	}
}

// DeviceIDs parses Devices (nil = every visible device).
func (c GPUVerifyConfig) DeviceIDs() ([]int, error) {
	if strings.TrimSpace(c.Devices) == "" {
		return nil, nil
	}
	var ids []int
	for _, f := range strings.Split(c.Devices, ",") {
		id, err := strconv.Atoi(strings.TrimSpace(f))
		if err != nil || id < 0 {
			return nil, fmt.Errorf("gpu-verify.devices: bad device id %q", f)
		}
		ids = append(ids, id)
	}
	return ids, nil
}

// Validate rejects values the library would refuse.
func (c GPUVerifyConfig) Validate() error {
	if _, err := c.DeviceIDs(); err != nil {
		return err
	}
	switch {
	case c.MaxBatch < 256:
		return fmt.Errorf("gpu-verify.max-batch must be >= 256, got %d", c.MaxBatch)
	case c.CPUBelow < 0, c.KeyLoadMin < 1, c.KeyCap < 1, c.EdKeyCap < 1, c.CacheEntries < 0:
		return fmt.Errorf("gpu-verify: negative or zero size in %+v", c)
	case c.CheckTxWindowTxs < 1 || c.CheckTxWindow < 0:
		return fmt.Errorf("gpu-verify: bad CheckTx window (%d txs, %v)", c.CheckTxWindowTxs, c.CheckTxWindow)
	}
	return nil
}

// GPUVerifyTemplate is the app.toml section (text/template over Config).
const GPUVerifyTemplate = `
###############################################################################
###                       GPU signature verification                        ###
###############################################################################

[gpu-verify]

# Route tx signature checks (x/auth ante, IBC commits) to the GPU verifier.
enable = {{ .GPUVerify.Enable }}

# HIP device ids, comma separated ("" = every visible device).
devices = "{{ .GPUVerify.Devices }}"

# Largest batch of one device call.
max-batch = {{ .GPUVerify.MaxBatch }}

# Batches with fewer signatures run on the CPU.
cpu-below = {{ .GPUVerify.CPUBelow }}

# Keep account keys parsed in GPU memory; loads only from key-load-min leaves.
keyed = {{ .GPUVerify.Keyed }}
key-load-min = {{ .GPUVerify.KeyLoadMin }}
key-cap = {{ .GPUVerify.KeyCap }}
ed-key-cap = {{ .GPUVerify.EdKeyCap }}

# Verdict cache entries (0 disables it).
cache-entries = {{ .GPUVerify.CacheEntries }}

# Concurrent CheckTx requests are pre-verified together: up to this many
# txs or this long after the first (a lone request never waits).
checktx-window-txs = {{ .GPUVerify.CheckTxWindowTxs }}
checktx-window = "{{ .GPUVerify.CheckTxWindow }}"

# Pre-verify each block before its DeliverTx loop.
preverify-blocks = {{ .GPUVerify.PreVerifyBlocks }}
`

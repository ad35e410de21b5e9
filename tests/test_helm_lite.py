"""testing/helm_lite.py: the Go text/template + sprig subset the chart uses,
with Go's semantics (checked on hand-computed expectations)."""
import pytest

from rocm_k8s_device_plugin_amd.testing.helm_lite import Renderer, TemplateError, _parse, _tokenize


def render(src, values=None, defines_src=""):
    defines = {}
    if defines_src:
        _parse(_tokenize(defines_src), defines)
    tree = _parse(_tokenize(src), defines)
    ctx = {"Values": values or {}, "Chart": {"Name": "c", "AppVersion": "1.2"}, "Release": {"Namespace": "ns"}}
    return Renderer(defines).run(tree, ctx, {"$": ctx})


def test_trim_markers_and_fields():
    assert render("a  {{- .Values.x -}}  b", {"x": "X"}) == "aXb"
    assert render("a {{ .Values.x }} b", {"x": 3.0}) == "a 3 b"          # float64 10 prints as 10
    assert render("{{ .Values.missing }}|") == "|"                      # <no value> -> ""
    assert render("{{/* a comment */}}ok") == "ok"


def test_if_else_truthiness():
    src = "{{ if .Values.a }}A{{ else if .Values.b }}B{{ else }}C{{ end }}"
    assert render(src, {"a": 1.0}) == "A"
    assert render(src, {"a": 0.0, "b": "x"}) == "B"
    assert render(src, {"a": "", "b": []}) == "C"
    assert render("{{ if and .Values.a (not .Values.b) }}y{{ end }}", {"a": True, "b": False}) == "y"


def test_pipelines_default_ternary_or():
    assert render('{{ .Values.tag | default .Chart.AppVersion }}', {"tag": ""}) == "1.2"
    assert render('{{ .Values.tag | default .Chart.AppVersion }}', {"tag": "t"}) == "t"
    assert render('{{ .Values.p | default (ternary 10 0 (or .Values.a .Values.b)) }}', {"p": 0.0, "b": True}) == "10"
    assert render('{{ printf "labeller-%s" .Chart.AppVersion }}') == "labeller-1.2"
    assert render('{{ ne .Values.k false }}', {"k": False}) == "false"


def test_range_with_variables_and_quote():
    assert render('{{- range .Values.args }}[{{ . | quote }}]{{- end }}', {"args": ["-a", "b c"]}) == '["-a"]["b c"]'
    assert render('{{- $x := .Values.v -}}{{ if $x }}{{ $x }}{{ end }}', {"v": "q"}) == "q"
    assert render('{{ with .Values.m }}{{ .k }}{{ end }}', {"m": {"k": "v"}}) == "v"


def test_include_nindent_toyaml():
    defs = '{{- define "lbl" -}}a: {{ .Chart.Name }}\nb: 1{{- end -}}'
    assert render('x:{{- include "lbl" . | nindent 2 }}', defines_src=defs) == "x:\n  a: c\n  b: 1"
    assert render('r: {{- toYaml .Values.r | nindent 2 }}', {"r": {}}) == "r:\n  {}"
    assert render('r: {{- toYaml .Values.r | nindent 2 }}', {"r": {"b": 1, "a": "x"}}) == "r:\n  a: x\n  b: 1"


def test_errors():
    with pytest.raises(TemplateError):
        render("{{ nosuchfunc 1 }}")
    with pytest.raises(TemplateError):
        render("{{ if .Values.a }}unterminated")


def test_chart_health_defaults_follow_the_measured_choice():
    """dp.liveness on: the probe server mode and the memory request come from
    profiles/r5/health_mode_choice.json (persistent; ~370Mi per GPU x 8); an
    explicit dp.resources wins; the raw health manifest says the same."""
    import json
    import os

    import yaml

    from rocm_k8s_device_plugin_amd.testing.helm_lite import rendered_objects
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    chart = os.path.join(repo, "helm", "amd-gpu")

    def dp(values):
        ds = [o for o in rendered_objects(chart, values)
              if o.get("kind") == "DaemonSet" and "labeller" not in o["metadata"]["name"]]
        return ds[0]["spec"]["template"]["spec"]["containers"][0]

    c = dp({"dp": {"liveness": {"enabled": True}}})
    assert "-liveness_mode=persistent" in c["args"] and c["resources"] == {"requests": {"memory": "3072Mi"}}
    assert "-prestart_liveness=true" in c["args"]
    assert "-prestart_liveness=false" in dp({"dp": {"liveness": {"enabled": True, "prestart": False}}})["args"]
    assert "-prestart_budget=5" in c["args"] and "-liveness_busy_deadline=0.05" in c["args"]
    tuned = dp({"dp": {"liveness": {"enabled": True, "prestartBudget": 8, "busyDeadline": 0.02}}})["args"]
    assert "-prestart_budget=8" in tuned and "-liveness_busy_deadline=0.02" in tuned
    assert dp({"dp": {"liveness": {"enabled": True, "mode": "spawn"}}})["args"].count("-liveness_mode=spawn") == 1
    assert dp({"dp": {"liveness": {"enabled": True}, "resources": {"limits": {"memory": "4Gi"}}}})["resources"] == \
        {"limits": {"memory": "4Gi"}}
    assert dp({})["resources"] == {}                                  # no liveness: no request (as upstream)
    choice = json.load(open(os.path.join(repo, "profiles", "r5", "health_mode_choice.json")))
    mem = [r["host_memory"] for r in choice["admissions_under_the_loop"].values()]
    probe_mib = max(m["children_rss_mb_max"] for m in mem)          # MiB per GPU (1-GPU box)
    daemon_mib = max(m["daemon_rss_mb_p50"] for m in mem)
    assert probe_mib <= 384 and 8 * probe_mib + daemon_mib <= 3 * 1024   # what the requests cover on 8 GPUs
    with open(os.path.join(repo, "k8s-ds-amdgpu-dp-health.yaml")) as f:
        man = yaml.safe_load(f)["spec"]["template"]["spec"]["containers"][0]
    assert "-liveness_mode=persistent" in man["args"] and man["resources"]["requests"]["memory"] == "3Gi"
    assert "-prestart_liveness=true" in man["args"]


def test_chart_device_count_and_config_file(tmp_path):
    """dp.deviceCount -> AMD_GPU_DEVICE_COUNT; dp.config -> a ConfigMap mounted at
    /etc/amdgpu/config.yaml with CONFIG_FILE_PATH (the upstream docs' recipe,
    docs/user-guide/configuration.md), read by the daemon as rendered."""
    import os
    import subprocess

    import yaml

    from rocm_k8s_device_plugin_amd.ops.native import PKG_DIR
    from rocm_k8s_device_plugin_amd.testing.fixtures import make_mi355x_node
    from rocm_k8s_device_plugin_amd.testing.helm_lite import rendered_objects
    chart = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "helm", "amd-gpu")
    objs = rendered_objects(chart, {"dp": {"deviceCount": 2, "config": {"gpu": {"device_count": 3}}}})
    cm = [o for o in objs if o.get("kind") == "ConfigMap"]
    ds = [o for o in objs if o.get("kind") == "DaemonSet" and "labeller" not in o["metadata"]["name"]][0]
    pod = ds["spec"]["template"]["spec"]
    c = pod["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env == {"AMD_GPU_DEVICE_COUNT": "2", "CONFIG_FILE_PATH": "/etc/amdgpu/config.yaml"}
    assert {"name": "config", "mountPath": "/etc/amdgpu", "readOnly": True} in c["volumeMounts"]
    assert len(cm) == 1 and {"name": "config", "configMap": {"name": cm[0]["metadata"]["name"]}} in pod["volumes"]
    assert yaml.safe_load(cm[0]["data"]["config.yaml"]) == {"gpu": {"device_count": 3}}
    # defaults render neither (as upstream)
    plain = [o for o in rendered_objects(chart, {}) if o.get("kind") == "DaemonSet"][0]
    assert "env" not in plain["spec"]["template"]["spec"]["containers"][0]
    assert not [o for o in rendered_objects(chart, {}) if o.get("kind") == "ConfigMap"]
    # the daemon reads what the chart mounts: the env beats the file, the file alone limits too
    fi = make_mi355x_node(tmp_path / "n")
    (tmp_path / "config.yaml").write_text(cm[0]["data"]["config.yaml"])
    exe = os.path.join(str(PKG_DIR), "bin", "mi355x-device-plugin")
    for extra, want in (({"AMD_GPU_DEVICE_COUNT": env["AMD_GPU_DEVICE_COUNT"]}, 2), ({}, 3)):
        e = {k: v for k, v in os.environ.items() if k != "AMD_GPU_DEVICE_COUNT"}
        e.update(extra, CONFIG_FILE_PATH=str(tmp_path / "config.yaml"))
        p = subprocess.run([exe, "-dry_run", "-sysfs_root", str(fi.sysfs), "-dev_root", str(fi.dev),
                            "-exporter_socket="], capture_output=True, text=True, timeout=30, env=e)
        assert p.returncode == 0, p.stderr[-500:]
        import json
        assert len(json.loads(p.stdout)["resources"]["amd.com/gpu"]["devices"]) == want


def test_chart_metrics_port_adds_probes():
    """dp.metricsPort: the daemon serves /metrics, /healthz and /readyz on it, and the DaemonSet's container gets a
    named port with a liveness probe on /healthz and a readiness probe on /readyz; without a port there are none
    (as upstream, which has no probes)."""
    import os

    from rocm_k8s_device_plugin_amd.testing.helm_lite import rendered_objects
    chart = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "helm", "amd-gpu")

    def dp(values):
        ds = [o for o in rendered_objects(chart, values)
              if o.get("kind") == "DaemonSet" and "labeller" not in o["metadata"]["name"]]
        return ds[0]["spec"]["template"]["spec"]["containers"][0]

    c = dp({"dp": {"metricsPort": 9400}})
    assert "-metrics_port=9400" in c["args"]
    assert c["ports"] == [{"name": "metrics", "containerPort": 9400}]
    assert c["livenessProbe"]["httpGet"] == {"path": "/healthz", "port": "metrics"}
    assert c["readinessProbe"]["httpGet"] == {"path": "/readyz", "port": "metrics"}
    # kubelet restarts the daemon after failureThreshold x periodSeconds of failed checks: well past the
    # daemon's own 60 s stall limit
    lp = c["livenessProbe"]
    assert lp["failureThreshold"] * lp["periodSeconds"] >= 60
    # the endpoint is served once the daemon is in its loop (after the first sweep): start-up has its own probe
    sp = c["startupProbe"]
    assert sp["httpGet"] == lp["httpGet"] and sp["failureThreshold"] * sp["periodSeconds"] >= 300
    plain = dp({})
    assert not {"ports", "startupProbe", "livenessProbe", "readinessProbe"} & set(plain)


def test_chart_labeller_metrics_port_adds_probes():
    """lbl.metricsPort: the labeller gets -metrics_port, a named port and probes on /healthz and /readyz."""
    import os

    from rocm_k8s_device_plugin_amd.testing.helm_lite import rendered_objects
    chart = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "helm", "amd-gpu")

    def lbl(values):
        ds = [o for o in rendered_objects(chart, dict(values, labeller={"enabled": True}))
              if o.get("kind") == "DaemonSet" and "labeller" in o["metadata"]["name"]]
        return ds[0]["spec"]["template"]["spec"]["containers"][0]

    c = lbl({"lbl": {"metricsPort": 9401}})
    assert "-metrics_port=9401" in c["args"]
    assert c["ports"] == [{"name": "metrics", "containerPort": 9401}]
    assert c["livenessProbe"]["httpGet"] == {"path": "/healthz", "port": "metrics"}
    assert c["readinessProbe"]["httpGet"] == {"path": "/readyz", "port": "metrics"}
    plain = lbl({})
    assert not {"ports", "startupProbe", "livenessProbe", "readinessProbe"} & set(plain)
    assert not any(a.startswith("-metrics_port") for a in plain["args"])

{{/* name helpers (same template names as upstream, so overrides keep working) */}}
{{- define "amd-gpu.name" -}}
{{- .Values.nameOverride | default .Chart.Name | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "amd-gpu.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- $n := include "amd-gpu.name" . -}}
{{- if contains $n .Release.Name -}}
{{- .Release.Name | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name $n | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}
{{- end -}}

{{- define "amd-gpu.chart" -}}
{{- printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "amd-gpu.selectorLabels" -}}
app.kubernetes.io/name: {{ include "amd-gpu.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end -}}

{{- define "amd-gpu.labels" -}}
helm.sh/chart: {{ include "amd-gpu.chart" . }}
{{ include "amd-gpu.selectorLabels" . }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end -}}

{{/* shared pod scheduling block: pull secrets, node selector, priority, tolerations */}}
{{- define "amd-gpu.podScheduling" -}}
{{- with .Values.imagePullSecrets }}
imagePullSecrets: {{ toYaml . | nindent 2 }}
{{- end }}
{{- if .Values.node_selector_enabled }}
{{- with .Values.node_selector }}
nodeSelector: {{ toYaml . | nindent 2 }}
{{- end }}
{{- end }}
priorityClassName: system-node-critical
{{- with .Values.tolerations }}
tolerations: {{ toYaml . | nindent 2 }}
{{- end }}
{{- end -}}
